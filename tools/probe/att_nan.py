import sys, torch
sys.path.insert(0, 'm2-tts_amd/src'); sys.path.insert(0, 'tests')
from m2amd import ops
from test_gpu_attention import make_qkv, ref_attention
for (B,N,H) in [(3,65,64),(3,63,64),(3,129,64),(3,200,64),(1,65,64),(3,65,32),(3,65,96)]:
    gen = torch.Generator().manual_seed(1000 * (H//2) + N)
    qkv = make_qkv(B, N, H, 2, "random", gen)
    got = ops.attention_core(qkv.cuda(), 2, None).cpu().double()
    ref = ref_attention(qkv, 2, None)
    nan = torch.isnan(got)
    print(B,N,H, 'nan count', int(nan.sum()), 'maxerr', float((got-ref)[~nan].abs().max()) if (~nan).any() else None)
    if nan.any():
        idx = nan.nonzero()
        print('   nan rows (b,q) sample', sorted(set((int(a),int(b_)) for a,b_,c in idx.tolist()))[:20], 'cols', sorted(set(int(c) for a,b_,c in idx.tolist()))[:70])
