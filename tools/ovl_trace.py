"""Timeline of the overlapped WAL scan's kernels from a rocprofv3 kernel trace.

usage: python3 tools/ovl_trace.py KERNEL_TRACE_CSV OUT_TXT

For the last few calls (each starts with wal_pipe_kernel<true>): every kernel
dispatched within 600 us of that start, with its start / end relative to it
(us) and its queue, so the overlap of phase A with the framing kernels and of
the class kernel with phase A's tail can be read off.
"""
import csv
import sys


def main(src, dst):
    rows = []
    with open(src, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id", "?")))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "wal_pipe_kernel" in r[2]]
    lines = []
    for si in starts[-3:]:
        t0 = rows[si][0]
        lines.append(f"call at {t0}")
        end = t0
        for k, (s, e, name, q) in enumerate(rows[si:]):
            if s - t0 > 600_000 or (k and "wal_pipe_kernel" in name):
                break
            end = max(end, e)
            short = name.split("(")[0][-60:]
            lines.append(f"  q{q:>3} {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {short}")
        lines.append(f"  span {(end - t0) / 1e3:.1f} us")
    open(dst, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[-12:]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
