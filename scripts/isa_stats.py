"""Per-kernel instruction counts from a device assembly file (diagnostic, CPU only).

usage: python scripts/isa_stats.py file.s [name-substring]
  (file.s from: hipcc <CXXFLAGS> --cuda-device-only -S csrc/X.hip -o file.s)
Prints, per kernel, static counts of scratch loads/stores, MFMAs, global stores/loads,
LDS ops and AGPR moves: a quick check for spills inside loops.
"""
import re
import sys

PATS = {"scratch_ld": r"\bscratch_load", "scratch_st": r"\bscratch_store", "mfma": r"\bv_mfma",
        "g_ld": r"\bglobal_load", "g_st": r"\bglobal_store", "ds_rd": r"\bds_read", "ds_wr": r"\bds_write",
        "acc_rd": r"\bv_accvgpr_read", "acc_wr": r"\bv_accvgpr_write", "s_waitcnt": r"\bs_waitcnt"}


def main():
    s = open(sys.argv[1]).read()
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r"^(\S+):\s*; @\S+\n(.*?)^\.Lfunc_end", s, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if want not in name:
            continue
        counts = " ".join(f"{k} {len(re.findall(p, body))}" for k, p in PATS.items())
        print(f"{name[:70]:70s} {counts}")


if __name__ == "__main__":
    main()
