"""Critical-path model of the device WAL scan's framing (wal_hist), round 6.

wal_hist walks every 32 KiB block's header chain with one thread per block
(log_reader.rs:271-331 framing); a wave holds 64 blocks and the launch ends
with its slowest wave, i.e. with the longest chains.  This replays the bench
log's framing (Random(301).skewed(17) records fragmented as
Writer::add_record does, log_writer.rs:62-110) on the CPU -- no bytes, only
positions -- and prices each hop: a header in a line no earlier hop of the
chain touched is an HBM round trip (HBM_US), one in a touched line an L2 hit
(L2_US); after TOUCH hops the rest of the block is in L2 (the touch);
LDS-window variants load up to NW windows of WB bytes per round trip and walk
them at LDS_US per hop.  Prints the slowest / 99th-percentile / mean wave for
each strategy.  The round-5 kernel measured 21.8 us against the model's
18.4 us for its strategy (launch and epilogue not modelled).
usage: python tools/r06/wal_chain_model.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "oracle"))
import wal_oracle as W  # noqa: E402  (test infrastructure: the bench log's record sizes)

HBM_US, L2_US, LDS_US, RT_US = 0.8, 0.25, 0.05, 1.0
B, H = W.BLOCK_SIZE, W.HEADER_SIZE


def bench_chains(target=262144 * 4096):
    r = W.Random(301)
    blocks, cur, off, tot = [], [], 0, 0
    while tot < target:
        n = r.skewed(17)
        tot += n
        left = n
        while True:
            if B - off < H:
                blocks.append(cur)
                cur, off = [], 0
            frag = min(left, B - off - H)
            cur.append(off)
            off += H + frag
            left -= frag
            if left == 0:
                break
    blocks.append(cur)
    return blocks


def touch_cost(ch, touch):
    lines, c, tf = set(), 0.0, None
    for k, p in enumerate(ch):
        ln = (p + 4) // 128
        c += L2_US if (tf is not None and p >= tf) or ln in lines else HBM_US
        lines.add(ln)
        if k + 1 == touch:
            tf = p
    return c


def window_wave(blocks, k0, nw, wb):
    t1, rem = 0.0, []
    for ch in blocks:
        t1 = max(t1, touch_cost(ch[:k0], 10 ** 9))
        if len(ch) > k0:
            rem.append(list(ch[k0:]))
    t = t1
    while rem:
        sel, rest, nxt, mx = rem[:nw], rem[nw:], [], 0.0
        for ch in sel:
            base, n = ch[0] & ~15, 0
            while n < len(ch) and ch[n] + 12 <= base + wb:
                n += 1
            n = max(n, 1)
            mx = max(mx, n * LDS_US)
            if n < len(ch):
                nxt.append(ch[n:])
        t += RT_US + mx
        rem = nxt + rest
    return t


def main():
    chains = bench_chains()
    nb = len(chains)
    cnt = np.array([len(c) for c in chains])
    print(f"blocks {nb}, records {cnt.sum()}, longest chain {cnt.max()}, blocks > 16 records {np.mean(cnt > 16):.3f}")
    waves = [chains[i:i + 64] for i in range(0, nb // 64 * 64, 64)]

    def report(name, costs):
        c = np.array(costs)
        print(f"{name:40s} slowest wave {c.max():5.1f} us  p99 {np.percentile(c, 99):5.1f}  mean {c.mean():5.1f}")
    for touch in (8, 16, 24, 10 ** 9):
        report(f"touch after {touch} hops" if touch < 10 ** 9 else "no touch",
               [max(touch_cost(c, touch) for c in w) for w in waves])
    for k0, nw, wb in ((16, 4, 4096), (8, 8, 4096), (6, 16, 2048), (2, 32, 1024)):
        report(f"LDS windows after {k0} hops, {nw} x {wb} B", [window_wave(w, k0, nw, wb) for w in waves])


if __name__ == "__main__":
    main()
