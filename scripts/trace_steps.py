"""Per-step GPU timeline from a rocprofv3 ``--kernel-trace`` CSV.

    python scripts/trace_steps.py <run_kernel_trace.csv> [anchor-substring] [last-k-steps]

A step starts at each dispatch whose name contains the anchor (default ``gram_``).  For the last k
steps prints every kernel's start offset / duration (us) relative to the step start and the
idle time between kernels, then the mean step period, busy time and idle time."""
import csv
import sys


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "gram_"
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    starts = [i for i, e in enumerate(ev) if anchor in e[2] and "reduce" not in e[2]]
    if len(starts) < 2:
        print("fewer than 2 anchored steps")
        return
    steps = [(starts[j], starts[j + 1]) for j in range(len(starts) - 1)]
    sel = steps[-k:]
    periods, busy = [], []
    for a, b in sel:
        t0 = ev[a][0]
        print(f"--- step @ {t0}")
        prev_end = t0
        bsum = 0
        for s, e, nm in ev[a:b]:
            gap = s - prev_end
            print(f"  +{(s - t0) / 1e3:8.1f}  {(e - s) / 1e3:8.1f} us  gap {gap / 1e3:7.1f}  {nm[:90]}")
            prev_end = max(prev_end, e)
            bsum += e - s
        periods.append(ev[b][0] - t0)
        busy.append(bsum)
    n = len(periods)
    print(f"mean period {sum(periods) / n / 1e3:.1f} us, busy {sum(busy) / n / 1e3:.1f} us, "
          f"idle {(sum(periods) - sum(busy)) / n / 1e3:.1f} us over {n} steps")


if __name__ == "__main__":
    main()
