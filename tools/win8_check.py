"""Host-side model of conv_wgrad_win8.hip's X ring and dZ staging (no GPU): for every split of
a launch geometry it replays the DMA schedule (prologue + 5 DMAs per wave per super-step,
DMA distance PD = 3: super-step S + 3 is issued at the top of iteration S) and checks that (1) a super-step never needs more than the 12 X blocks
its 4 waves issue, (2) every ring row a super-step's tap reads holds that frame row when it
is read (loaded, not yet overwritten), (3) the transposing reads of a 32-lane half hit 64
distinct LDS banks.  Usage: python tools/win8_check.py [B] [splits...]"""
import sys

WF, FP, SPB, XR = 21, 448, 13, 1024
PD = 3


def g0(s):
    b = s // SPB
    return b * FP + WF + 32 * (s - b * SPB)


def swz(slot):
    return (slot >> 2) & 3


def check(B, splits):
    TS = B * SPB // 4
    worst_blocks = 0
    for z in range(splits):
        s0, s1 = z * TS // splits, (z + 1) * TS // splits
        if s0 >= s1:
            continue
        ring = {}                       # slot -> frame row
        lo = (g0(4 * s0) - 22) & ~15
        hi = (g0(4 * s0 + 3) + 54 + 15) & ~15
        for r in range(lo, hi):
            ring[r & (XR - 1)] = r
        loaded_hi = hi
        pending = []                    # DMAs issued, landed at the next barrier

        def issue(Sn):
            nonlocal loaded_hi, worst_blocks
            lo0 = (g0(4 * Sn) - 22) & ~15
            lo_ = max(lo0, loaded_hi)
            hi_ = (g0(4 * Sn + 3) + 54 + 15) & ~15
            nblk = (hi_ - lo_) >> 4
            worst_blocks = max(worst_blocks, nblk)
            assert nblk <= 12, (Sn, nblk)
            rows = []
            for k in range(12):
                r0 = lo_ + 16 * (k if k < nblk else 0)
                rows += list(range(r0, r0 + 16))
            loaded_hi = hi_
            return rows
        for pp in range(1, PD):
            if s0 + pp < s1:
                pending.append(issue(s0 + pp))
        for S in range(s0, s1):
            inflight = set()
            if S + PD < s1:
                pending.append(issue(S + PD))
            # every pending DMA may land while S is read: none may overwrite S's rows
            for rows in pending:
                inflight |= {r & (XR - 1) for r in rows}
            for r in range(4):
                for t in range(9):
                    off = (t // 3 - 1) * WF + (t % 3 - 1)
                    for row in range(g0(4 * S + r) + off, g0(4 * S + r) + off + 32):
                        slot = row & (XR - 1)
                        assert ring.get(slot) == row, (z, S, r, t, row, ring.get(slot))
                        if slot in inflight:
                            assert all(rr == row for rows in pending for rr in rows
                                       if (rr & (XR - 1)) == slot), ("overwrite", S, row)
            # bottom of iteration S: S + 1's DMA has landed
            if pending:
                for row in pending.pop(0):
                    ring[row & (XR - 1)] = row
    return worst_blocks


def banks():
    """(3) one ds_read_b64_tr_b8: lanes 0-31 = rows base + 0..15 (two groups of 8), chunk c
    (16 B of the 64-B row), lane pair halves 8 B each -> 64 banks of 4 B must be distinct."""
    for base in range(512):
        for c in range(4):
            seen = set()
            for lane in range(32):
                g, li = lane >> 4, lane & 15
                q, p = li >> 1, li & 1
                slot = (base + 8 * g + q) & (XR - 1)
                addr = slot * 64 + ((c ^ swz(slot)) * 16) + 8 * p
                for w in range(2):
                    bank = (addr // 4 + w) % 64
                    assert bank not in seen, (base, c, lane)
                    seen.add(bank)


if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    banks()
    for sp in [int(x) for x in sys.argv[2:]] or [1, 2, 3, 6, 12, 25, 64]:
        print(f"B={B} splits={sp}: ok, max X blocks per super-step {check(B, sp)}")
