"""CPU checks of the librosa-0.10 restatement used as the f4 checker
(oracle/audio_oracle.py).  librosa is not installed, so these pin the
restatement to the published algorithm's known properties instead:
perfect reconstruction of the Hann/hop-256 STFT (COLA), the Slaney mel
scale's anchor points and the area normalisation of the filters, a pure tone
landing in the band that contains it, power_to_db's floor."""
import numpy as np

import audio_oracle as ao


def test_stft_istft_roundtrip():
    x = np.random.default_rng(0).standard_normal(10000).astype(np.float32)
    S = ao.stft(x, 1024, 256, 1024)
    assert S.shape == (513, 1 + 10000 // 256)
    y = ao.istft(S, 1024, 256, 1024)
    assert len(y) == 256 * (S.shape[1] - 1)
    assert np.abs(y - x[:len(y)]).max() < 2e-6


def test_stft_matches_direct_dft():
    x = np.random.default_rng(1).standard_normal(3000).astype(np.float32)
    S = ao.stft(x, 512, 128, 512)
    w = ao.hann_periodic(512).astype(np.float64)
    xp = np.pad(x, 256).astype(np.float64)
    t = 5
    frame = xp[t * 128:t * 128 + 512] * w
    k = np.arange(257)[:, None]
    n = np.arange(512)[None, :]
    ref = (frame[None, :] * np.exp(-2j * np.pi * k * n / 512)).sum(1)
    assert np.abs(S[:, t] - ref).max() < 1e-4


def test_slaney_mel_scale_and_filters():
    assert abs(ao.hz_to_mel(1000.0) - 15.0) < 1e-12           # linear part: 1000 / (200/3)
    assert abs(ao.mel_to_hz(ao.hz_to_mel(4321.0)) - 4321.0) < 1e-9
    W = ao.mel_filterbank(22050, 1024, 64, 0, 11025)
    assert W.shape == (64, 513) and (W >= 0).all()
    # slaney norm: each triangle has area 1 in Hz (weights * bin spacing summed ~ 1)
    df = 22050 / 1024
    areas = W.sum(1) * df
    assert np.all(np.abs(areas[8:] - 1) < 0.05)


def test_tone_lands_in_its_band_and_db_floor():
    t = np.arange(22050) / 22050
    for f in (300.0, 2500.0):
        y = np.sin(2 * np.pi * f * t).astype(np.float32)
        mel = ao.compute_mel_spectrogram(y)
        band = int(np.argmax(mel[:, 40]))
        edges = ao.mel_to_hz(np.linspace(ao.hz_to_mel(0), ao.hz_to_mel(11025), 66))
        assert edges[band] <= f <= edges[band + 2]
    db = ao.power_to_db(np.array([[1.0, 1e-12, 1e-3]], dtype=np.float32))
    assert db.max() == 0.0 and db.min() == -80.0 and abs(db[0, 2] + 30.0) < 1e-4


def test_nnls_restatement_blocks_and_start():
    """librosa.util.nnls restated: 1024-column blocks for 64 float32 bands,
    each an L-BFGS-B problem on the block-normalised objective; in the
    normalised mel range its convergence test passes at the clipped-pinv
    start, so the result IS that start (what the GPU reproduces)."""
    A = ao.mel_filterbank(22050, 1024, 64, 0, 11025.0)
    rng = np.random.default_rng(2)
    mel = rng.uniform(-1, 1, (64, 1100)).astype(np.float32)
    M = np.power(10.0, 0.1 * (mel + 1) / 2).astype(np.float32)
    assert ao.nnls_block_columns(A, M) == 1024
    X, info = ao.nnls_lbfgs(A, M, return_info=True)
    assert len(info) == 2 and all(nit == 0 for nit, _ in info)
    X0 = np.clip(np.linalg.pinv(A) @ M, 0, None)
    assert np.array_equal(X, X0.astype(np.float32))
    assert ao.nnls_projected_gradient_norm(A, X0[:, :1024], M[:, :1024]) <= 1e-5
    # far outside the range the start is not stationary and L-BFGS-B iterates
    big = (rng.standard_normal((64, 40)) * 20).astype(np.float32)
    Mb = np.power(10.0, 0.1 * (big + 1) / 2).astype(np.float32)
    Xb, ib = ao.nnls_lbfgs(A, Mb, return_info=True)
    assert ib[0][0] > 0
    assert ao.nnls_objective(A, Xb, Mb) < ao.nnls_objective(A, np.clip(np.linalg.pinv(A) @ Mb, 0, None), Mb)
