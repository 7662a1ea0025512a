#!/usr/bin/env python3
"""Timeline summary of a rocprofv3 kernel trace (rocpd SQLite: ``rocprofv3 --kernel-trace -d D
-o run -- ...`` writes D/run_results.db): over the span of the kernels matching --span
(default: the GPU JPEG Huffman decode, i.e. the store-image pass), per kernel family the summed
time and the union of busy time (sum > union = launches overlapped), the hardware queue of every
stream, and how often a matching kernel ran concurrently with another of its family.

  python tools/kernel_overlap.py gpurun_out/prof/run_results.db [--span jpeg_huff]
"""
import argparse
import collections
import sqlite3


def union_ms(iv):
    iv = sorted(iv)
    if not iv:
        return 0.0
    busy, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return (busy + ce - cs) / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--span", default="jpeg_huff")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, queue_id, stream_id from kernels order by start").fetchall()
    sp = [r for r in rows if a.span in r[0]]
    if not sp:
        raise SystemExit(f"no kernel matches {a.span!r}")
    t0, t1 = sp[0][1], sp[-1][2]
    win = [r for r in rows if t0 <= r[1] <= t1]
    print(f"span of {a.span}: {(t1 - t0) / 1e6:.1f} ms, {len(win)} kernels")
    fam = collections.defaultdict(list)
    for r in win:
        fam["jpeg" if "jpeg" in r[0] else "model"].append((r[1], r[2]))
    fam[a.span] = [(r[1], r[2]) for r in sp]
    for k, iv in fam.items():
        print(f"  {k:>12}: {len(iv):6d} launches, sum {sum(e - s for s, e in iv) / 1e6:8.1f} ms, "
              f"union {union_ms(iv):8.1f} ms")
    q = collections.Counter((r[4], r[3], "jpeg" if "jpeg" in r[0] else "model") for r in win)
    print("  stream -> queue:", ", ".join(f"s{s}->q{qq} {k} x{n}" for (s, qq, k), n in sorted(q.items())))
    over = sum(1 for x, y in zip(sp, sp[1:]) if y[1] < x[2])
    print(f"  consecutive {a.span} launches that overlapped: {over} of {len(sp) - 1}")


if __name__ == "__main__":
    main()
