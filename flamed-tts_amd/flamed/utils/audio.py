"""WAV I/O without librosa / soundfile (absent offline): scipy.io.wavfile + linear resampling."""
import numpy as np
from scipy.io import wavfile
from scipy.signal import resample_poly


def load_wav(path: str, sr: int = 16000) -> np.ndarray:
    """Mono float32 in [-1, 1] at `sr` (librosa.load(path, sr=sr)[0] equivalent)."""
    rate, data = wavfile.read(path)
    if data.dtype.kind == "i":
        data = data.astype(np.float32) / float(np.iinfo(data.dtype).max)
    elif data.dtype.kind == "u":
        data = (data.astype(np.float32) - 128.0) / 128.0
    data = data.astype(np.float32)
    if data.ndim > 1:
        data = data.mean(axis=1)
    if rate != sr:
        g = np.gcd(rate, sr)
        data = resample_poly(data, sr // g, rate // g).astype(np.float32)
    return data


def write_wav(path: str, wav: np.ndarray, sr: int = 16000) -> None:
    """float32 WAV (soundfile.write(path, wav, sr) equivalent)."""
    wavfile.write(path, sr, np.asarray(wav, dtype=np.float32))
