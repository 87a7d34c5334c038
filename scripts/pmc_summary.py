"""Per-kernel PMC summary of one or more rocprofv3 --pmc passes over the same
command (diagnostic; writes the JSON the round's profiles/ keeps).

usage: python scripts/pmc_summary.py OUT.json PASS_DIR [PASS_DIR ...]

For every kernel name: dispatch count, mean duration (from the counter rows'
start/end timestamps), mean of every counter per dispatch, and derived values:
  hbm_bytes   = 2 * FETCH_SIZE + WRITE_SIZE (KB -> B; FETCH_SIZE doubled for
                gfx950's half-counted 16-B-per-lane reads, MI355X_MICROARCH.md
                HBM section; Infinity-Cache hits included)
  hbm_GBs     = hbm_bytes / duration
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
  l2_hit_rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  clock_GHz   = GRBM_GUI_ACTIVE / 8 XCDs / duration
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").strip()


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(dict)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                k = short(r["Kernel_Name"])
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                durs[k][(path, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    res = {}
    for k, cs in vals.items():
        e = {"dispatches": max(len(v) for v in cs.values()),
             "mean_ns": sum(durs[k].values()) / max(len(durs[k]), 1)}
        for c, v in cs.items():
            e[c] = sum(v) / len(v)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
            e["hbm_GBs"] = e["hbm_bytes"] / e["mean_ns"] if e["mean_ns"] else None
        if "SQ_VALU_MFMA_BUSY_CYCLES" in e and e.get("GRBM_GUI_ACTIVE"):
            e["mfma_busy"] = e["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * e["GRBM_GUI_ACTIVE"] / 8)
        if e.get("GRBM_GUI_ACTIVE") and e["mean_ns"]:
            e["clock_GHz"] = e["GRBM_GUI_ACTIVE"] / 8 / e["mean_ns"]
        if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e and e["TCC_HIT_sum"] + e["TCC_MISS_sum"] > 0:
            e["l2_hit_rate"] = e["TCC_HIT_sum"] / (e["TCC_HIT_sum"] + e["TCC_MISS_sum"])
        res[k] = e
    res = dict(sorted(res.items(), key=lambda kv: -kv[1]["mean_ns"] * kv[1]["dispatches"]))
    json.dump({"source": dirs, "kernels": res}, open(out, "w"), indent=1)
    for k, e in list(res.items())[:8]:
        extra = {x: round(e[x], 3) if isinstance(e.get(x), float) else e.get(x)
                 for x in ("hbm_GBs", "mfma_busy", "l2_hit_rate", "clock_GHz") if x in e}
        print(f"{k[:48]:48s} n={e['dispatches']:3d} {e['mean_ns'] / 1e3:10.1f} us {extra}")


if __name__ == "__main__":
    main()
