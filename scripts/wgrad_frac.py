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
    mac_hidden = sum(o * i for o, i in LAYERS[conf] if min(o, i) > 64)
    # the backward chain's workgroups (64 samples each, any wave count) -> samples (SB x R x N) of the pass; the
    # weight-gradient dispatches that follow it: the batched kernel and (ABI 16) the thin layers' launches
    passes = {4 * 512 * 96: "fine", 4 * 512 * 64: "coarse"}
    pending, cur, out = None, None, {"fine": [], "coarse": []}

    def flush():
        if cur is not None and cur["batched"] > 0:
            out[passes[cur["M"]]].append((cur["batched"] + cur["thin"], cur["batched"], cur["thin"], cur["M"]))

    for r in rows:
        n = r["Kernel_Name"]
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        if "field_bwd" in n:
            flush()
            cur = None
            pending = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) * 64
            if pending in passes:
                cur = {"M": pending, "batched": 0.0, "thin": 0.0}
        elif cur is not None and "thin_wgrad_kernel" in n:
            cur["thin"] += ms
        elif cur is not None and "weight_grad_kernel" in n:
            cur["batched"] += ms
    flush()
    for k, v in out.items():
        if not v:
            continue
        v.sort()
        tot, bat, thin, M = v[len(v) // 2]
        tf_all = 2.0 * M * mac / (tot * 1e-3) / 1e12
        line = (f"{conf} {k:6s} pass: M = {M} rows, {len(v)} passes, median {tot:.3f} ms = {tf_all:.1f} TFLOP/s "
                f"(fp32-equivalent, every layer) = {tf_all / X3_PEAK:.3f} of the {X3_PEAK:.1f} TF x3 peak")
        if thin > 0:
            tf_b = 2.0 * M * mac_hidden / (bat * 1e-3) / 1e12
            line += (f"; batched kernel {bat:.3f} ms on the hidden layers = {tf_b / X3_PEAK:.3f}, thin launches "
                     f"{thin * 1e3:.0f} us")
        print(line)


if __name__ == "__main__":
    main()
