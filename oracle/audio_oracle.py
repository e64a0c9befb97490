"""CPU oracle for the mel-feature / Griffin-Lim path.

TEST INFRASTRUCTURE ONLY (like m2tts_oracle.py): nothing in the product path
imports it; tests/ use it as the checker.

The reference (src/utils/audio.py:45-151) calls librosa (requirements.txt:6
pins librosa>=0.10.0), which is NOT installed in this image, so the reference
cannot be run here: this file restates librosa 0.10's published algorithms
for exactly the calls and defaults the reference makes, and the parity of
that restatement with librosa itself is UNPINNED (no librosa output exists
in /root/reference to check it against).  What it restates:

  compute_mel_spectrogram (audio.py:45-98)
    librosa.feature.melspectrogram(y, sr, n_fft, hop_length, win_length,
      n_mels, fmin, fmax, power=2.0) with librosa 0.10 defaults:
      window='hann' (periodic, scipy.signal.get_window fftbins=True),
      center=True, pad_mode='constant' (zero padding of n_fft // 2 per side),
      filters.mel(htk=False, norm='slaney')  (Slaney mel scale, area norm)
    librosa.power_to_db(S, ref=np.max, amin=1e-10, top_db=80.0)
    then 2 (x - min) / (max - min) - 1
  mel_to_audio (audio.py:101-151)
    (mel + 1) / 2, librosa.db_to_power, librosa.feature.inverse.mel_to_audio
      (n_iter=32, power=2.0): mel_to_stft = nnls(mel_basis, M) ** (1/power)
      (librosa.util.nnls: pinv init clipped at 0, then per block of <= 1024
      columns scipy fmin_l_bfgs_b with bounds >= 0 and m = n_fft // 2 + 1
      on the objective normalised by the block's size), then griffinlim(momentum=0.99,
      init='random') and istft; finally / max|audio|.
  The random phase init of griffinlim is an input here (init_angles), so a
  run is reproducible and the GPU path can be checked on the same angles.
"""
from __future__ import annotations

import numpy as np

AMIN = 1e-10
TOP_DB = 80.0


def hann_periodic(n: int) -> np.ndarray:
    """scipy.signal.get_window('hann', n, fftbins=True)."""
    k = np.arange(n, dtype=np.float64)
    return (0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)).astype(np.float32)


def hz_to_mel(f):
    """librosa.hz_to_mel(htk=False): Slaney - linear below 1 kHz, log above."""
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, mels)


def mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filterbank(sr: int, n_fft: int, n_mels: int, fmin: float, fmax: float) -> np.ndarray:
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk=False, norm='slaney') -> [n_mels, n_fft//2+1] f32."""
    fftfreqs = np.fft.rfftfreq(n_fft, 1.0 / sr)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    w = np.zeros((n_mels, len(fftfreqs)), dtype=np.float64)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    w *= enorm[:, None]
    return w.astype(np.float32)


def stft(y: np.ndarray, n_fft: int, hop: int, win_length: int) -> np.ndarray:
    """librosa.stft(center=True, pad_mode='constant', window='hann') of a 1-D
    float32 signal -> complex64 [n_fft//2+1, frames]."""
    win = np.zeros(n_fft, dtype=np.float32)
    lpad = (n_fft - win_length) // 2
    win[lpad:lpad + win_length] = hann_periodic(win_length)
    yp = np.pad(y.astype(np.float32), n_fft // 2, mode="constant")
    n_frames = 1 + (len(yp) - n_fft) // hop
    idx = np.arange(n_fft)[None, :] + hop * np.arange(n_frames)[:, None]
    frames = yp[idx] * win[None, :]
    return np.fft.rfft(frames.astype(np.float64), axis=1).astype(np.complex64).T


def istft(S: np.ndarray, n_fft: int, hop: int, win_length: int, length=None) -> np.ndarray:
    """librosa.istft(center=True, window='hann'): windowed inverse frames,
    overlap-add, divided by the window's sum of squares where it exceeds
    tiny(float32), then the n_fft // 2 centre padding trimmed."""
    win = np.zeros(n_fft, dtype=np.float32)
    lpad = (n_fft - win_length) // 2
    win[lpad:lpad + win_length] = hann_periodic(win_length)
    n_frames = S.shape[1]
    frames = np.fft.irfft(S.T.astype(np.complex128), n=n_fft, axis=1).astype(np.float32) * win[None, :]
    out_len = n_fft + hop * (n_frames - 1)
    y = np.zeros(out_len, dtype=np.float32)
    wss = np.zeros(out_len, dtype=np.float32)
    w2 = win.astype(np.float32) ** 2
    for t in range(n_frames):
        y[t * hop:t * hop + n_fft] += frames[t]
        wss[t * hop:t * hop + n_fft] += w2
    nz = wss > np.finfo(np.float32).tiny
    y[nz] /= wss[nz]
    y = y[n_fft // 2:]
    if length is None:
        y = y[:out_len - n_fft]
    else:
        y = y[:length]
    return y


def power_to_db(S: np.ndarray) -> np.ndarray:
    """librosa.power_to_db(S, ref=np.max, amin=1e-10, top_db=80)."""
    S = np.asarray(S, dtype=np.float32)
    ref = np.max(S)
    log_spec = 10.0 * np.log10(np.maximum(AMIN, S))
    log_spec -= 10.0 * np.log10(np.maximum(AMIN, ref))
    return np.maximum(log_spec, log_spec.max() - TOP_DB).astype(np.float32)


def compute_mel_spectrogram(audio, sample_rate=22050, n_fft=1024, hop_length=256, win_length=1024, n_mels=64,
                            fmin=0, fmax=None) -> np.ndarray:
    """src/utils/audio.py:45-98 -> [n_mels, frames] float32 in [-1, 1]."""
    if fmax is None:
        fmax = sample_rate // 2
    S = np.abs(stft(np.asarray(audio, dtype=np.float32), n_fft, hop_length, win_length)) ** 2
    mel = mel_filterbank(sample_rate, n_fft, n_mels, fmin, fmax) @ S.astype(np.float32)
    db = power_to_db(mel)
    return (2 * (db - db.min()) / (db.max() - db.min()) - 1).astype(np.float32)


MAX_MEM_BLOCK = 2 ** 8 * 2 ** 10  # librosa.util.utils.MAX_MEM_BLOCK (256 KiB)


def nnls_block_columns(A: np.ndarray, B: np.ndarray) -> int:
    """librosa.util.nnls: columns per L-BFGS-B block, MAX_MEM_BLOCK //
    (prod(B.shape[:-1]) * A.itemsize) (1024 for 64 float32 mel bands)."""
    return max(1, int(MAX_MEM_BLOCK // (int(np.prod(B.shape[:-1])) * A.itemsize)))


def nnls_lbfgs(A: np.ndarray, B: np.ndarray, return_info: bool = False):
    """librosa.util.nnls (0.10) for a 2-D B: X0 = max(0, pinv(A) B) (float32,
    as A), then per block of nnls_block_columns columns scipy's
    fmin_l_bfgs_b(bounds >= 0, m = A.shape[1], default pgtol 1e-5 / factr 1e7)
    on librosa's _nnls_obj: (1 / B_blk.size) * 0.5 ||A X - B_blk||^2 and its
    gradient (1 / B_blk.size) A^T (A X - B_blk), from X0's columns.  The
    normalisation by B.size makes the stopping test scale-free: for every
    mel in the reference's normalised range the projected gradient at X0 is
    below pgtol and L-BFGS-B returns X0 itself (nit 0).  return_info adds
    the per-block scipy (nit, task)."""
    import scipy.optimize
    x_init = np.clip(np.linalg.pinv(A) @ B, 0, None)
    n_col = nnls_block_columns(A, B)
    x = x_init.copy()
    info = []
    for s0 in range(0, B.shape[-1], n_col):
        s1 = min(s0 + n_col, B.shape[-1])
        Bb = B[:, s0:s1]
        x0 = x_init[:, s0:s1]
        shape, scale = x0.shape, 1.0 / Bb.size

        def obj(v, shape=shape, Bb=Bb, scale=scale):
            v = v.reshape(shape)
            diff = A @ v - Bb
            return scale * 0.5 * np.sum(diff ** 2), (scale * (A.T @ diff)).ravel()

        v, _, d = scipy.optimize.fmin_l_bfgs_b(obj, x0.ravel(), bounds=[(0, None)] * x0.size, m=A.shape[1])
        x[:, s0:s1] = v.reshape(shape)
        info.append((int(d["nit"]), str(d["task"])))
    x = x.astype(A.dtype)
    return (x, info) if return_info else x


def nnls_projected_gradient_norm(A: np.ndarray, X: np.ndarray, B: np.ndarray) -> float:
    """L-BFGS-B's convergence measure (projgr) at X for one block: the
    infinity norm of the projected gradient of librosa's scaled objective
    (lower bound 0: g if g < 0 else min(x, g))."""
    Xd, Ad = X.astype(np.float64), A.astype(np.float64)
    g = (Ad.T @ (Ad @ Xd - B.astype(np.float64))) / B.size
    pg = np.where(g < 0, g, np.minimum(Xd, g))
    return float(np.abs(pg).max()) if pg.size else 0.0


def nnls_objective(A, X, B) -> float:
    return float(0.5 * np.sum((A.astype(np.float64) @ X.astype(np.float64) - B.astype(np.float64)) ** 2))


def griffin_lim(S: np.ndarray, init_angles: np.ndarray, n_iter: int, n_fft: int, hop: int, win_length: int,
                momentum: float = 0.99) -> np.ndarray:
    """librosa.griffinlim(S, n_iter, momentum, init='random') with the random
    phases given as init_angles (complex unit values, S.shape)."""
    angles = init_angles.astype(np.complex64).copy()
    eps = np.finfo(np.float32).tiny
    rebuilt = np.zeros_like(angles)
    for _ in range(n_iter):
        tprev = rebuilt
        inverse = istft(S * angles, n_fft, hop, win_length)
        rebuilt = stft(inverse, n_fft, hop, win_length)
        angles = rebuilt - (momentum / (1 + momentum)) * tprev
        angles = (angles / (np.abs(angles) + eps)).astype(np.complex64)
    return istft(S * angles, n_fft, hop, win_length)


def mel_to_audio(mel_spec, init_angles, sample_rate=22050, n_fft=1024, hop_length=256, win_length=1024, n_iter=32,
                 n_mels=None, nnls=nnls_lbfgs):
    """src/utils/audio.py:101-151 with the griffinlim phases given."""
    mel = (np.asarray(mel_spec, dtype=np.float32) + 1) / 2
    M = np.power(10.0, 0.1 * mel).astype(np.float32)            # db_to_power(ref=1)
    W = mel_filterbank(sample_rate, n_fft, n_mels or M.shape[0], 0, sample_rate / 2.0)
    S = np.power(nnls(W, M), 0.5).astype(np.float32)            # mel_to_stft, power=2
    audio = griffin_lim(S, init_angles, n_iter, n_fft, hop_length, win_length)
    m = np.max(np.abs(audio))
    return (audio / m if m > 0 else audio).astype(np.float32), S
