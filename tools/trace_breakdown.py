#!/usr/bin/env python
"""Per-kernel and per-launch breakdown of the timed forwards in a rocprofv3 kernel trace.

    python tools/trace_breakdown.py TRACE.csv --forwards 5:3 [--out profiles/x.txt]

--forwards TOTAL:TIMED: the trace holds TOTAL forwards that launch the same kernel sequence
(calibration forwards excluded by counting from the end), the last TIMED of them are the timed
steps.  The window starts at the first dispatch of the timed forwards (found by splitting the
dispatch list at the period of the last forward's sequence).  Prints the time per kernel name
over the window and one forward's launches in order (name, grid, workgroup, duration), which
attributes every layer of the network.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--forwards", default="5:3", help="TOTAL:TIMED forwards at the end of the trace")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    total, timed = (int(x) for x in a.forwards.split(":"))
    with open(a.trace, newline="") as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))

    def key(r):
        return (r["Kernel_Name"], r.get("Grid_Size_X", r.get("Grid_Size", "")))
    # the host's read-backs after the timed region (counter copies) are not part of a forward
    while rows and rows[-1]["Kernel_Name"].startswith("__amd_rocclr_copy"):
        rows.pop()
    # period = dispatches per forward: the smallest p for which the last TIMED forwards repeat
    n = len(rows)
    period = None
    for p in range(1, n // timed + 1):
        if all(key(rows[n - 1 - i]) == key(rows[n - 1 - p - i]) for i in range(p * (timed - 1))):
            period = p
            break
    if period is None:
        raise SystemExit("no periodic forward sequence found")
    win = rows[n - timed * period:]
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    span = int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])
    busy = sum(dur(r) for r in win)
    by = collections.defaultdict(lambda: [0, 0])
    for r in win:
        nm = r["Kernel_Name"].split("(")[0][:90]
        by[nm][0] += dur(r)
        by[nm][1] += 1
    out = [f"trace {a.trace}", f"dispatches per forward {period}; window = last {timed} forwards: "
           f"span {span / 1e6 / timed:.3f} ms/forward, kernel busy {busy / 1e6 / timed:.3f} ms/forward", "",
           "per kernel (ms per forward, % of busy, dispatches per forward):"]
    for nm, (t, c) in sorted(by.items(), key=lambda kv: -kv[1][0]):
        out.append(f"  {t / 1e6 / timed:8.3f} ms  {100.0 * t / busy:5.1f} %  {c // timed:4d}  {nm}")
    out += ["", "one forward, in launch order (us, grid x, workgroup x, name):"]
    for r in win[-period:]:
        out.append(f"  {dur(r) / 1e3:9.1f}  {r.get('Grid_Size_X', r.get('Grid_Size', '')):>9}  "
                   f"{r.get('Workgroup_Size_X', r.get('Workgroup_Size', '')):>4}  {r['Kernel_Name'].split('(')[0][:80]}")
    text = "\n".join(out)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
