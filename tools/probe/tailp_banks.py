#!/usr/bin/env python3
"""LDS bank-conflict check for the pipelined tail's B-fragment reads and
epilogue writes (vocoder_tailp.hip): every K-slot list of tp::kslot,
ds_read_b128 / ds_write_b64 lane groups from MI355X_MICROARCH.md (LDS table).
Padded-row layouts (the earlier RS 144..208 strides) and, with --swizzle, the
current unpadded 64-B hi / lo planes with octet o of row r at
16 * (o ^ ((r >> 1) & 3)).

    python tools/probe/tailp_banks.py
"""
GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
          list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
          list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]



def F(dq):
    return [(0, dq, o) for o in range(4)]


K = {  # (layer, mb): [kb][g] = (res, dq, octet); pad slots read (0, g) against zero weights
    (0, 0): [F(0), F(-1)], (0, 1): [F(1), F(0)],
    (1, 0): [F(0), [(0, -1, 2), (0, -1, 3), (0, 0, 2), (0, 0, 3)]], (1, 1): [F(0), [(0, 1, 0), (0, 1, 1), (0, 0, 2), (0, 0, 3)]],
    (2, 0): [F(0), [(0, -1, 2), (0, -1, 3), (1, 0, 0), (1, 0, 1)]],
    (2, 1): [F(0), [(0, 1, 0), (0, 1, 1), (1, 0, 2), (1, 0, 3)]],
    (3, 0): [F(0), [(0, -1, 2), (0, -1, 3), (0, 0, 2), (0, 0, 3)]], (3, 1): [F(0), [(0, 1, 0), (0, 1, 1), (0, 0, 2), (0, 0, 3)]],
    (4, 0): [[(0, -1, 3), (0, 0, 0), (0, 0, 1), (0, 0, 2)]],
    (4, 1): [[(0, 0, 1), (0, 0, 2), (0, 0, 3), (0, 1, 0)]],
    (6, 0): [F(0), [(0, -1, 3), (0, 1, 0), (0, 0, 2), (0, 0, 3)]],
}


def reads(rs, verbose):
    worst = 1
    for key, kbs in K.items():
        for kb in kbs:
            for lo in (0, 64):
                for grp in GROUPS:
                    slots = []
                    for lane in grp:
                        li, g = lane & 15, lane >> 4
                        res, dq, oc = kb[g]
                        row = li + dq - (2 if res else 1)
                        addr = row * rs + oc * 16 + lo + (64 * rs if res else 0)
                        slots.append((addr // 16) % 16)
                    c = max(slots.count(x) for x in set(slots))
                    if c > 1 and verbose:
                        print(f"  RS {rs}: {c}-way read conflict {key} kb {kb} {'lo' if lo else 'hi'}")
                    worst = max(worst, c)
    return worst


def writes_b64(rs):
    worst = 1
    for g in range(4):
        banks = []
        for li in range(16):
            a = li * rs + 8 * g
            banks += [(a // 4) % 32, (a // 4 + 1) % 32]
        worst = max(worst, max(banks.count(x) for x in set(banks)))
    return worst


def writes_b128(rs):
    """Octet-wide stores (one 16-B chunk per lane after a permlane16 swap): 8 x 8 contiguous lanes."""
    worst = 1
    for base in range(0, 64, 8):
        banks = []
        for lane in range(base, base + 8):
            li, g = lane & 15, lane >> 4
            a = li * rs + 16 * g
            banks += [(a // 4 + i) % 32 for i in range(4)]
        worst = max(worst, max(banks.count(x) for x in set(banks)))
    return worst


def swizzled():
    """Current layout: every fragment read and 8-row b128 store conflict free."""
    worst_r = worst_w = 1
    for key, kbs in K.items():
        for kb in kbs:
            for r0 in range(64):
                for grp in GROUPS:
                    v = []
                    for lane in grp:
                        li, g = lane & 15, lane >> 4
                        res, dq, oc = kb[g]
                        r = (r0 + li + dq - (2 if res else 1)) % 64
                        v.append((r * 64 + 16 * (oc ^ ((r >> 1) & 3))) // 16 % 16)
                    worst_r = max(worst_r, max(v.count(x) for x in set(v)))
    for r0 in range(64):
        for o in range(4):
            v = [(((r0 + li) % 64) * 64 + 16 * (o ^ ((((r0 + li) % 64) >> 1) & 3))) // 16 % 8 for li in range(8)]
            worst_w = max(worst_w, max(v.count(x) for x in set(v)))
    return worst_r, worst_w


if __name__ == "__main__":
    import sys
    if "--swizzle" in sys.argv:
        r, w = swizzled()
        print(f"swizzled 64-B planes: reads {r}-way, ds_write_b128 {w}-way")
        sys.exit(0)
    for rs in (144, 160, 176, 208):
        print(f"RS {rs}: reads {reads(rs, False)}-way, ds_write_b64 {writes_b64(rs)}-way, "
              f"ds_write_b128 {writes_b128(rs)}-way")
