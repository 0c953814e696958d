"""WAV I/O without librosa / soundfile (absent offline): scipy.io.wavfile + polyphase resampling
(librosa.load resamples with soxr; outputs at a different input rate differ slightly)."""
import numpy as np
from scipy.io import wavfile
from scipy.signal import resample_poly


def load_wav(path: str, sr: int = 16000) -> np.ndarray:
    """Mono float32 in [-1, 1] at `sr` (librosa.load(path, sr=sr)[0] equivalent)."""
    rate, data = wavfile.read(path)
    if data.dtype.kind == "i":
        data = data.astype(np.float32) / float(2 ** (8 * data.dtype.itemsize - 1))  # libsndfile scaling
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
    """16-bit PCM WAV, as `soundfile.write(path, wav, sr)` writes float data by default (subtype PCM_16,
    samples clipped to [-1, 1] and scaled by 32767)."""
    pcm = np.rint(np.clip(np.asarray(wav, dtype=np.float64), -1.0, 1.0) * 32767.0).astype(np.int16)
    wavfile.write(path, sr, pcm)
