from .facodec import (FACodecDecoder, FACodecEncoder, EncoderBlock, SnakeBeta, ResidualUnit,  # noqa: F401
                      DecoderBlock, WNConv1d, WNConvTranspose1d)
from .alias_free_torch import Activation1d  # noqa: F401
