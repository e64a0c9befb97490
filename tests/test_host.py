"""Host-side checks that need no GPU: the C-ABI library loads and exports every
symbol include/m2tts_hip.h declares, the weight table matches the reference
state_dict layout, argument errors are reported, and the product path refuses
CPU tensors (no CPU fallback)."""
import ctypes
import re

import pytest
import torch

from conftest import ROOT, golden


def header_functions():
    text = (ROOT / "include" / "m2tts_hip.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|size_t|const char\s*\*)\s*(m2_\w+)\s*\(", text, re.M)))


def test_library_exports_every_header_symbol():
    from m2amd import _lib
    lib = _lib.load()
    funcs = header_functions()
    assert len(funcs) >= 25
    for f in funcs:
        assert hasattr(lib, f), f"{f} declared in include/m2tts_hip.h but not exported"
        assert f in _lib._SIGNATURES, f"{f} has no ctypes signature in m2amd/_lib.py"
    assert lib.m2_abi_version() == 1


def test_abi_argument_errors_are_reported():
    from m2amd import _lib
    from m2amd.runtime import make_config
    lib = _lib.load()
    bad = make_config(256, 64, 64, 2, 2, 3, 128, 1000)  # 64 % 3 != 0
    assert lib.m2_weight_count(ctypes.byref(bad)) < 0
    assert b"invalid config" in lib.m2_last_error()
    good = make_config(256, 64, 64, 2, 2, 2, 128, 1000)
    buf = ctypes.create_string_buffer(8)
    assert lib.m2_weight_name(ctypes.byref(good), 0, buf, 8) == -1  # buffer too small
    assert lib.m2_weight_name(ctypes.byref(good), 10 ** 6, ctypes.create_string_buffer(64), 64) == -1
    assert lib.m2_workspace_bytes(None, 1, 1, 1) == 0
    out = ctypes.c_void_p()
    assert lib.m2_model_create(ctypes.byref(bad), None, 0, None, ctypes.byref(out)) == -1
    with pytest.raises(_lib.M2Error, match="bad argument"):
        _lib.call("m2_linear", None, None, None, None, None, None, 0, 1, 8, 8, None, None)


@pytest.mark.parametrize("cfg", [dict(), dict(hidden_dim=96, mel_channels=80, text_encoder_layers=3, decoder_layers=3,
                                               vocoder_channels=256),
                                 dict(vocab_size=100, hidden_dim=32, mel_channels=32, text_encoder_layers=1,
                                      decoder_layers=1, vocoder_channels=64)])
def test_weight_table_matches_state_dict(cfg):
    from models.tts_model import M2TTSModel
    from m2amd.runtime import weight_names
    m = M2TTSModel(**cfg)
    sd = m.state_dict()
    names = weight_names(m._m2_cfg)
    assert [n for n, _ in names] == list(sd.keys())  # same keys, same order as the reference state_dict
    assert all(sd[n].numel() == k for n, k in names)


def test_seeded_init_reproduces_reference_weights():
    """torch.manual_seed(1234); M2TTSModel() == the reference's init (fixture
    weights were made by the reference; only the pinned projection differs)."""
    from models.tts_model import M2TTSModel
    torch.manual_seed(1234)
    sd = M2TTSModel().state_dict()
    w = golden("weights_s1")
    pinned = "duration_predictor.predictor.projection"
    for k in sd:
        if not k.startswith(pinned):
            assert torch.equal(sd[k], torch.from_numpy(w[k])), k
    u = golden("weights_s1_unpinned_proj")
    assert torch.equal(sd[pinned + ".weight"], torch.from_numpy(u["weight"]))


def test_cpu_tensors_fail_loudly():
    from models.components import MultiHeadAttention
    from models.tts_model import M2TTSModel, SimpleVocoder
    m = M2TTSModel().eval()
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        m.inference(torch.zeros(1, 4, dtype=torch.long), torch.tensor([4]))
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        m(torch.zeros(1, 4, dtype=torch.long))
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        SimpleVocoder()(torch.zeros(1, 64, 3))
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        MultiHeadAttention(32, 2)(torch.zeros(1, 3, 32))


def test_get_model_size_counts():
    from models.tts_model import M2TTSModel
    info = M2TTSModel().get_model_size()
    assert info["total_params"] == 321154  # measured on the reference
    assert info["components"]["vocoder"]["total"] == 142209
    info2 = M2TTSModel(hidden_dim=96, mel_channels=80, text_encoder_layers=3, decoder_layers=3,
                       vocoder_channels=256).get_model_size()
    assert info2["total_params"] == 1066610


def test_vocoder_halo_is_the_receptive_field():
    """The streamed vocoder's halo (C constant, Python constant) equals the
    receptive field propagated through the reference's layer stack."""
    import sys
    sys.path.insert(0, str(ROOT / "tools" / "probe"))
    import receptive_field
    from m2amd import _lib
    from models.tts_model import VOCODER_HALO
    assert receptive_field.halo_frames() == (3, 3)
    assert _lib.load().m2_vocoder_halo_frames() == VOCODER_HALO == 3


def test_oracle_vocoder_chunked_within_reorder_noise():
    """The oracle (reference ATen ops) on a 3-frame-halo window gives the same
    centre samples up to fp32 reordering noise (7e-7)."""
    import m2tts_oracle as orc
    from conftest import golden_state
    sd = golden_state("s1")
    mel = torch.randn(1, 64, 40, generator=torch.Generator().manual_seed(5))
    full = orc.vocoder(sd, mel)
    f0, f1 = 12, 25
    win = orc.vocoder(sd, mel[:, :, f0 - 3:f1 + 3])
    assert float((win[:, :, 64 * 3:64 * (3 + f1 - f0)] - full[:, :, 64 * f0:64 * f1]).abs().max()) <= 2e-6


def test_bench_flop_model():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.vocoder_flops_per_sample(128, 64) == 14896.0
    assert bench.vocoder_flops_per_sample(256, 80) == 58336.0
    assert sum(bench.vocoder_kernel_flops_per_frame(128, 64)) == 14896 * 64


def test_range_policy_default_and_env_validation(monkeypatch):
    """New handles get the "fallback" policy (no non-finite audio returned for
    finite inputs) unless M2_RANGE_POLICY names another; a bad value is an
    error naming the variable, at configuration time."""
    from m2amd.runtime import default_range_policy
    from models.tts_model import M2TTSModel
    monkeypatch.delenv("M2_RANGE_POLICY", raising=False)
    assert default_range_policy() == "fallback"
    monkeypatch.setenv("M2_RANGE_POLICY", "report")
    assert default_range_policy() == "report"
    monkeypatch.setenv("M2_RANGE_POLICY", "fallbak")
    with pytest.raises(ValueError, match="M2_RANGE_POLICY"):
        default_range_policy()
    with pytest.raises(ValueError, match="range policy"):
        M2TTSModel().set_range_policy("nope")
