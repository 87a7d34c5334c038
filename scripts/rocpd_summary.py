"""Diagnostic: summarise a rocprofv3 results database (ROCm 7 writes rocpd SQLite by default): per kernel name the
dispatch count, mean duration and the mean of every collected counter per dispatch.
usage: python scripts/rocpd_summary.py <results.db> [name-substring ...]"""
import collections
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    want = sys.argv[2:]
    names = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    disp = collections.defaultdict(list)
    ev = {}
    for kid, start, end, eid in c.execute("select kernel_id, start, end, event_id from rocpd_kernel_dispatch"):
        disp[names[kid]].append(end - start)
        ev[eid] = names[kid]
    pmc_names = {r[0]: r[1] for r in c.execute("select id, name from rocpd_info_pmc")}
    pmc = collections.defaultdict(lambda: collections.defaultdict(float))
    for eid, pid, val in c.execute("select event_id, pmc_id, value from rocpd_pmc_event"):
        if eid in ev:
            pmc[ev[eid]][pmc_names[pid]] += val
    for k, d in sorted(disp.items(), key=lambda kv: -sum(kv[1])):
        if want and not any(w in k for w in want):
            continue
        print(f"{k[:90]}: {len(d)} dispatches, mean {sum(d) / len(d) / 1e3:.1f} us")
        for p, v in sorted(pmc[k].items()):
            print(f"    {p:28s} {v / len(d):16.1f} per dispatch")


if __name__ == "__main__":
    main()
