"""Per-launch durations of one kernel from a rocprofv3 --kernel-trace CSV, split into the
untimed warmup launches and the timed ones (bench.py's --warmup / --steps), so the bench
line's roofline `avg_launch_ms` can be reproduced from profiles/ without the cold calls.

    python tools/timed_launches.py TRACE.csv KERNEL_SUBSTRING WARMUP STEPS
"""
import csv
import sys


def main():
    path, kname, warm, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rows = [r for r in csv.DictReader(open(path)) if kname in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    name = rows[0]["Kernel_Name"] if rows else kname
    print("%s launch durations (us) in launch order (%s); the first %d are the untimed warmup"
          % (name, path, warm))
    print(" ".join("%.1f" % x for x in d))
    t = d[warm:warm + steps]
    if t:
        print("timed %d: mean %.1f us, min %.1f, max %.1f; all %d: mean %.1f us"
              % (len(t), sum(t) / len(t), min(t), max(t), len(d), sum(d) / len(d)))


if __name__ == "__main__":
    main()
