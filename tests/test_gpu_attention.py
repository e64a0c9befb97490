"""Flash attention kernel (transformer.hip attention_split_kernel) against a
float64 torch reference of the reference's MultiHeadAttention core
(components.py:60-90: softmax(q k^T / sqrt(hd), masked_fill(-1e9)) v).

Covers every head_dim instance (16/32/48/64), both query-tile variants,
ragged lengths around the 64-key chunk and 128-query block edges, masked
and unmasked forms, and score patterns that drive the unmasked path's lazy
rescaling: a ramp whose scores grow by more than the rescale threshold in
every chunk (the base moves on every chunk), a falling ramp (it never moves
after the first chunk), and large random logits.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 2e-5  # observed <= 5e-7 on N(0, 1) data; split-f16 products at fp32 accuracy


def ref_attention(qkv, heads, mask):
    B, N, H3 = qkv.shape
    H = H3 // 3
    hd = H // heads
    q, k, v = qkv.double().view(B, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    s = q @ k.transpose(-1, -2) / hd ** 0.5
    if mask is not None:
        s = s.masked_fill(~mask[:, None, None, :], -1e9)
    return (s.softmax(-1) @ v).transpose(1, 2).reshape(B, N, H)


def make_qkv(B, N, H, heads, pattern, gen):
    qkv = torch.randn(B, N, 3 * H, generator=gen)
    if pattern == "large":
        qkv[..., : 2 * H] *= 4.0
    elif pattern in ("ramp", "fall"):
        hd = H // heads
        u = torch.randn(hd, generator=gen)
        u /= u.norm()
        j = torch.arange(N, dtype=torch.float32)
        # score(query, key j) ~ sqrt(hd) * c_j / sqrt(hd) = c_j: +0.25 per key (16 per 64-key chunk)
        c = 0.25 * (j if pattern == "ramp" else (N - 1 - j))
        q = u.repeat(heads) * hd ** 0.5
        qkv[..., :H] = q + 0.01 * qkv[..., :H]
        qkv[..., H:2 * H] = (c[:, None] * u.repeat(heads)[None, :])[None] + 0.01 * qkv[..., H:2 * H]
    return qkv


@pytest.mark.parametrize("hd", [16, 32, 48, 64])
@pytest.mark.parametrize("N", [1, 63, 65, 129, 511])
@pytest.mark.parametrize("masked", [False, True])
def test_attention_shapes(gpu, hd, N, masked):
    from m2amd import ops
    heads, H = 2, 2 * hd
    gen = torch.Generator().manual_seed(1000 * hd + N)
    B = 3
    qkv = make_qkv(B, N, H, heads, "random", gen)
    mask = None
    if masked:
        lens = torch.randint(1, N + 1, (B,), generator=gen)
        mask = torch.arange(N)[None, :] < lens[:, None]
    got = ops.attention_core(qkv.to(gpu), heads, None if mask is None else mask.to(gpu)).cpu().double()
    assert float((got - ref_attention(qkv, heads, mask)).abs().max()) <= TOL


@pytest.mark.parametrize("pattern", ["ramp", "fall", "large"])
@pytest.mark.parametrize("hd,B,N", [(32, 64, 500), (32, 2, 500), (48, 2, 700), (64, 1, 300)])
def test_attention_rescale_patterns(gpu, pattern, hd, B, N):
    """(32, 64, 500) takes the two-query-tile variant (grid of >= 256 workgroups)."""
    from m2amd import ops
    heads, H = 2, 2 * hd
    gen = torch.Generator().manual_seed(hd * N + B)
    qkv = make_qkv(B, N, H, heads, pattern, gen)
    got = ops.attention_core(qkv.to(gpu), heads, None).cpu().double()
    ref = ref_attention(qkv, heads, None)
    assert torch.isfinite(got).all()
    # logits reach ~125 (180 in base 2) in the ramps: a score carries an
    # absolute error of ~2^-22 of that (split-f16 products, fp32 accumulate),
    # ~4e-5 relative on the weights -> the bound scales with it
    assert float((got - ref).abs().max()) <= 1e-4 * max(1.0, float(ref.abs().max()))


def test_attention_long_form(gpu):
    """T = 2600 (the long-form decoder): 41 chunks per utterance."""
    from m2amd import ops
    gen = torch.Generator().manual_seed(7)
    qkv = make_qkv(2, 2600, 96, 2, "random", gen)
    got = ops.attention_core(qkv.to(gpu), 2, None).cpu().double()
    assert float((got - ref_attention(qkv, 2, None)).abs().max()) <= TOL


@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("N", [257, 500])
def test_attention_wide_grid_head_dim_32(gpu, masked, N):
    """B=64, hd 32: grids of >= 256 workgroups take the two-query-tile
    variant (128 queries per workgroup), masked and unmasked."""
    from m2amd import ops
    heads, H, B = 2, 64, 64
    gen = torch.Generator().manual_seed(N + masked)
    qkv = make_qkv(B, N, H, heads, "random", gen)
    mask = None
    if masked:
        lens = torch.randint(1, N + 1, (B,), generator=gen)
        mask = torch.arange(N)[None, :] < lens[:, None]
    got = ops.attention_core(qkv.to(gpu), heads, None if mask is None else mask.to(gpu)).cpu().double()
    assert float((got - ref_attention(qkv, heads, mask)).abs().max()) <= TOL
