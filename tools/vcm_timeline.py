"""Print the last N kernel dispatches of a rocprofv3 --kernel-trace database (ms from the first
dispatch, duration in us, stream/queue, name): the VCM overlapped schedule has no photon pass, so
tools/timeline_summary.py does not apply."""
import glob
import sqlite3
import sys


def main():
    root = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    db = sorted(glob.glob(root + '/**/*.db', recursive=True))[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name,start,end,stream_id,queue_id from kernels order by start"))
    t0 = rows[0][1]
    for name, s, e, st, q in rows[-n:]:
        print(f"{(s - t0) / 1e6:10.3f} {(e - s) / 1e3:9.1f}us st{st} q{q} {name[:70]}")


if __name__ == "__main__":
    main()
