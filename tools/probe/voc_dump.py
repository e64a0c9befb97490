"""Stage2 vocoder audio of seeded mel at several B x T shapes, saved per shape
(gpurun_out/<tag>_<BxT>.npy) with the library named by M2TTS_HIP_LIB, so two
builds' tilings can be checked bit for bit (`--compare tagA tagB`).

    python tools/probe/voc_dump.py dump <tag> 8x500 16x262 ...
    python tools/probe/voc_dump.py compare <tagA> <tagB> 8x500 16x262 ...
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
OUT = ROOT / "gpurun_out"


def dump(tag, shapes):
    sys.path.insert(0, str(ROOT))
    import torch
    import bench

    m = bench.fixture_model(bench.STAGE2, torch.device("cuda:0"))
    for sh in shapes:
        b, t = (int(v) for v in sh.split("x"))
        g = torch.Generator().manual_seed(77 + b * 10007 + t)
        mel = torch.randn(b, bench.STAGE2["mel_channels"], t, generator=g).cuda()
        with torch.no_grad():
            a = m.vocoder(mel)
        torch.cuda.synchronize()
        np.save(OUT / f"{tag}_{sh}.npy", a.float().cpu().numpy())
        print(tag, sh, tuple(a.shape), flush=True)


def compare(ta, tb, shapes):
    bad = 0
    for sh in shapes:
        a, b = np.load(OUT / f"{ta}_{sh}.npy"), np.load(OUT / f"{tb}_{sh}.npy")
        same = a.shape == b.shape and np.array_equal(a, b)
        diff = float(np.abs(a - b).max()) if a.shape == b.shape else float("nan")
        print(f"{sh}: {'bit-identical' if same else 'DIFFERENT'} (max |diff| {diff:.3g})", flush=True)
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    OUT.mkdir(exist_ok=True)
    if sys.argv[1] == "dump":
        dump(sys.argv[2], sys.argv[3:])
    else:
        compare(sys.argv[2], sys.argv[3], sys.argv[4:])
