#!/usr/bin/env python3
"""Concurrency summary of a rocprofv3 --kernel-trace database of the pipelined bench (tools/gpu.sh timeline):
the last N photon-pass iterations, how much of that wall time 0/1/2/3 kernels run, and each kernel's wall time
per iteration.  Usage: timeline_summary.py run_results.db [iterations]"""
import collections
import sqlite3
import sys


def main():
    db, n_it = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12
    c = sqlite3.connect(db)
    rows = [(r[0].split("(")[0].replace("void orx::", "").strip(), int(r[1]), int(r[2]), r[3])
            for r in c.execute("select name, start, end, stream_id from kernels order by start")]
    photon = [r for r in rows if r[0].startswith("k_ppm_photon")]
    # the timed window: from the start of the n_it-th last photon pass to the end of the last kernel before
    # the serial leg (the bench line ran with --no-serial-pass-times, so that is the last kernel)
    t0 = photon[-n_it][1]
    t1 = max(r[2] for r in rows)
    win = [(n, max(s, t0), min(e, t1), st) for n, s, e, st in rows if e > t0 and s < t1]
    ev = sorted([(s, 1) for _, s, _, _ in win] + [(e, -1) for _, _, e, _ in win])
    cover = collections.Counter()
    cur, last = 0, t0
    for t, d in ev:
        cover[cur] += t - last
        cur += d
        last = t
    total = t1 - t0
    print(f"# last {n_it} iterations: {total / n_it / 1e6:.3f} ms per iteration")
    for k in sorted(cover):
        print(f"{k} kernels running: {100.0 * cover[k] / total:5.1f} % of the time")
    per = collections.defaultdict(float)
    stream = {}
    for n, s, e, st in win:
        base = n.split("(")[0]
        per[base] += (e - s) / 1e6 / n_it
        stream[base] = st
    print("# wall time per iteration each kernel is running (ms), stream")
    for k, v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"  {k:40s} {v:6.3f}  stream {stream[k]}")


if __name__ == "__main__":
    main()
