"""Flamed-TTS, MI355X-native flow-matching hot path (drop-in for the reference `flamed` package).

`from flamed import Flamed` works as in the reference; submodules import lazily so the HIP
denoiser / duration generator / FaCodec decoder can be used on their own.
"""


def __getattr__(name):
    if name == "Flamed":
        from .models.flamed import Flamed
        return Flamed
    raise AttributeError(name)
