"""Weight-gradient kernel's fraction of the x3 peak in a train.py step, per dispatch, from a rocprofv3
kernel trace of `bench.py --mode train` (the fine- and coarse-pass calls alternate after their backward
chains). usage: python scripts/wgrad_frac.py TRACE.csv [default_mv|default]"""
import csv
import sys

X3_PEAK = 2500.0 / 3.0                                   # TFLOP/s: fp16 dense MFMA / 3 products
LAYERS = {  # (out, in) of every layer whose dW the kernel forms: blocks x (fc_0, fc_1), lin_z, lin_in, lin_out
    "default_mv": [(512, 512)] * (2 * 5 + 3) + [(512, 44), (4, 512)],
    "default": [(512, 512)] * (2 * 3 + 3) + [(512, 44), (4, 512)],
}


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    conf = sys.argv[2] if len(sys.argv) > 2 else "default_mv"
    mac = sum(o * i for o, i in LAYERS[conf])
    # the backward chain's workgroups (64 samples each, any wave count) -> samples (SB x R x N) of the pass
    passes = {4 * 512 * 96: "fine", 4 * 512 * 64: "coarse"}
    pending, out = None, {"fine": [], "coarse": []}
    for r in rows:
        n = r["Kernel_Name"]
        if "field_bwd" in n:
            pending = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) * 64
        elif "weight_grad_kernel" in n and pending in passes:
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            M = pending
            out[passes[pending]].append((ms, 2.0 * M * mac / (ms * 1e-3) / 1e12, M))
    for k, v in out.items():
        v.sort()
        ms, tf, M = v[len(v) // 2]
        print(f"{conf} {k:6s} pass: M = {M} rows, {len(v)} dispatches, median {ms:.3f} ms = {tf:.1f} TFLOP/s "
              f"(fp32-equivalent) = {tf / X3_PEAK:.3f} of the {X3_PEAK:.1f} TF x3 peak")


if __name__ == "__main__":
    main()
