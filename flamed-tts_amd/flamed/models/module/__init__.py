from .transformer import Encoder, Decoder, FFTBlock  # noqa: F401
