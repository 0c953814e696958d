from .facodec import FACodecDecoder, SnakeBeta, ResidualUnit, DecoderBlock, WNConv1d, WNConvTranspose1d  # noqa: F401
from .alias_free_torch import Activation1d  # noqa: F401
