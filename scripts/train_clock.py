"""Per training kernel (by grid size): shader clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch time, and MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), medians over the dispatches of a
rocprofv3 --pmc counter-collection CSV. usage: python scripts/train_clock.py FILE.csv"""
import collections
import csv
import sys

KERNELS = ("weight_grad_kernel", "field_x3_kernel", "field_bwd_x3_kernel")


def main():
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(sys.argv[1])):
        name = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
        if name is None:
            continue
        d = per[(name, r["Grid_Size"] if "Grid_Size" in r else r.get("Grid_Size_X", ""), r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    groups = collections.defaultdict(list)
    for (name, grid, _), d in per.items():
        if "GRBM_GUI_ACTIVE" in d and d["ns"] > 0:
            cyc = d["GRBM_GUI_ACTIVE"] / 8.0
            groups[(name, grid)].append((d["ns"] / 1e6, cyc / d["ns"], d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * 1024)))
    for (name, grid), v in sorted(groups.items()):
        v.sort()
        ms, ghz, busy = v[len(v) // 2]
        print(f"{name:22s} grid {grid:>9s}: {len(v)} dispatches, median {ms:.3f} ms, {ghz:.3f} GHz, MFMA busy {busy:.3f}")


if __name__ == "__main__":
    main()
