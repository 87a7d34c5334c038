"""One training step's kernel timeline from a rocprofv3 --kernel-trace CSV (diagnostic): every dispatch of the
last complete step in order, with its duration and the idle gap before it, plus per-kernel totals over that step.
Steps are delimited by a marker kernel that runs once per step (default: the march backward's parameter reduce).

usage: python scripts/step_timeline.py TRACE.csv [MARKER_SUBSTRING] [N_STEPS_TO_SKIP_FROM_END]"""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name).replace("void ", "")
    return name[:70]


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "raymarch_grads_reduce"
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(ends) < skip + 2:
        raise SystemExit(f"found {len(ends)} '{marker}' dispatches; need {skip + 2}")
    a, b = ends[-skip - 2] + 1, ends[-skip - 1] + 1
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = int(step[-1]["End_Timestamp"])
    busy, prev_end = 0, t0
    tot = collections.defaultdict(lambda: [0, 0])
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = max(0, s - prev_end)
        busy += e - s
        k = short(r["Kernel_Name"])
        tot[k][0] += 1
        tot[k][1] += e - s
        print(f"{(s - t0) / 1e3:9.1f} us  +{gap / 1e3:7.1f} gap  {(e - s) / 1e3:8.1f} us  "
              f"grid {r.get('Grid_Size_X', '?'):>8s}  {k}")
        prev_end = max(prev_end, e)
    print(f"\nstep span {(t1 - t0) / 1e3:.1f} us, kernel time {busy / 1e3:.1f} us, {len(step)} dispatches")
    for k, (n, ns) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{ns / 1e3:9.1f} us  {n:4d}x  {k}")


if __name__ == "__main__":
    main()
