#!/usr/bin/env python
"""Summarise rocprofv3 CSV output for the approx GEMM op (profiles/ evidence).

    python tools/prof_summary.py --trace DIR/..._kernel_trace.csv --stats DIR/..._kernel_stats.csv \
        [--pmc DIR/..._counter_collection.csv ...] --timed-launches N --out profiles/rocprof_r01

Writes <out>.json (machine-readable) and <out>.txt (human-readable).  The timed-region
average takes the LAST N dispatches of --kernel (the dominant kernel, gemm_f8mx_kernel; bench.py's
timed steps come last); op_avg_ns adds every kernel of one approx op (--op-kernels: operand
pre-decodes, the GEMM, the split-K reduce, the gated exact kernel) over the same window -- the
quantity bench.py times with HIP events.  PMC counters are averaged per dispatch of --kernel;
HBM traffic per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 bytes (rocprofv3's KB units).  On
gfx950 FETCH_SIZE reports half the bytes of coalesced buffer loads: MI355X_MICROARCH.md §HBM for
16 B / lane, and tools/fetch_cal.hip (profiles/fetch_cal_r02.txt) for this kernel's 4 B / lane
A-word loads as well (1 GiB read -> 512 MiB FETCH_SIZE for both widths); WRITE_SIZE is exact for
4 and 16 B / lane stores.
"""
FETCH_CAL = 2.0  # bytes read per FETCH_SIZE byte (tools/fetch_cal.hip)
import argparse
import collections
import csv
import json

OP_KERNELS = ("xm_decode_a,xm_decode_b,tt_decode_b,v5mx_decode_b,gemm_f8mx_kernel,gemm_v5mx_kernel,gemm_tt_kernel,"
              "gemm_tt16_kernel,gemm_fast_kernel,splitk_reduce_kernel,gemm_exact_kernel")


def read_csv(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--stats")
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--timed-launches", type=int, default=0,
                    help="the last N dispatches of --kernel are the timed ones (0: use --forwards)")
    ap.add_argument("--forwards", default="",
                    help="TRACE_FORWARDS:TIMED[,PMC_FORWARDS:TIMED]: every forward launches --kernel equally "
                         "often, so the timed dispatches are the last total x TIMED / FORWARDS")
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    ap.add_argument("--pmc-json", default="", help="also write the per-launch PMC summary bench.py reads")
    ap.add_argument("--kernel", default="gemm_f8mx_kernel")
    ap.add_argument("--arch", default="resnet18", help="bench workload the PMC passes ran (bench.py keys on it)")
    ap.add_argument("--E", type=int, default=4)
    ap.add_argument("--M", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="images per step of the profiled bench run")
    ap.add_argument("--op-kernels", default=OP_KERNELS)
    ap.add_argument("--pmc-launches", type=int, default=0,
                    help="average PMC counters over the last N dispatches of --kernel per file (0 = all)")
    a = ap.parse_args()
    KERNEL = a.kernel

    trace = read_csv(a.trace)
    rows = [r for r in trace if KERNEL in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fw = [tuple(int(x) for x in f.split(":")) for f in a.forwards.split(",") if f]
    n_timed = a.timed_launches or (len(rows) * fw[0][1] // fw[0][0] if fw else len(rows))
    timed = rows[-n_timed:]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
    # the op window: from the first timed dispatch's preceding pre-decode (if any) to the end
    t0 = int(timed[0]["Start_Timestamp"]) if timed else 0
    pre = [int(r["Start_Timestamp"]) for r in trace if "xm_decode_a" in r["Kernel_Name"] and int(r["Start_Timestamp"]) < t0]
    w0 = max(pre) if pre else t0
    opk = [k for k in a.op_kernels.split(",") if k]
    op_rows = [r for r in trace if int(r["Start_Timestamp"]) >= w0 and any(k in r["Kernel_Name"] for k in opk)]
    op_ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in op_rows)
    res = dict(kernel=KERNEL, all_dispatches=len(rows), timed_dispatches=len(timed),
               timed_avg_ns=sum(durs) / max(1, len(durs)), timed_total_ns=sum(durs),
               op_avg_ns=op_ns / max(1, len(timed)), op_kernels=opk,
               vgpr=timed[-1]["VGPR_Count"] if timed else None, lds=timed[-1]["LDS_Block_Size"] if timed else None,
               note=a.note)
    if a.stats:
        res["stats_top"] = [dict(name=r["Name"][:120], calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]),
                                 pct=float(r["Percentage"])) for r in read_csv(a.stats)[:8]]
    # per counter file: the LAST --pmc-launches dispatches of KERNEL (the PMC runs' timed steps;
    # averaging over every dispatch would mix in the calibration pass's smaller launches)
    counters = collections.defaultdict(list)
    for p in a.pmc:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in read_csv(p):
            if KERNEL in r.get("Kernel_Name", ""):
                per[int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))][r["Counter_Name"]] += float(r["Counter_Value"])
        keep = a.pmc_launches or (len(per) * fw[1][1] // fw[1][0] if len(fw) > 1 else 0)
        for d in sorted(per)[-keep:] if keep > 0 else sorted(per):
            for k, v in per[d].items():
                counters[k].append(v)
    if counters:
        res["pmc_avg_per_dispatch"] = {k: sum(v) / len(v) for k, v in counters.items()}
        pm = res["pmc_avg_per_dispatch"]
        if "FETCH_SIZE" in pm and "WRITE_SIZE" in pm:
            res["bytes_per_launch"] = (FETCH_CAL * pm["FETCH_SIZE"] + pm["WRITE_SIZE"]) * 1024.0
            res["traffic_note"] = "(2 x FETCH_SIZE + WRITE_SIZE) x 1024: FETCH_SIZE calibrated at 1/2 (tools/fetch_cal.hip)"
        if "SQ_INSTS_VALU" in pm and "SQ_WAVES" in pm:
            res["valu_instr_per_wave"] = pm["SQ_INSTS_VALU"] / pm["SQ_WAVES"]
    if counters and a.pmc_json:
        pm = res["pmc_avg_per_dispatch"]
        pj = dict(source="rocprofv3 --kernel-trace --pmc (separate passes per counter group, "
                         f"--kernel-include-regex {KERNEL}) on bench.py --steps 2 --warmup 1",
                  note=f"per {KERNEL} dispatch, averaged; FETCH_SIZE/WRITE_SIZE in KB (x1024 = bytes); "
                       "bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: FETCH_SIZE reads half the bytes of "
                       "4- and 16-B-per-lane buffer loads (tools/fetch_cal.hip, MI355X_MICROARCH.md HBM section)",
                  arch=a.arch, E=a.E, M=a.M, batch=a.batch)
        pj["kernel"] = KERNEL
        if "FETCH_SIZE" in pm and "WRITE_SIZE" in pm:
            pj.update(kernel=KERNEL, bytes_per_launch=(FETCH_CAL * pm["FETCH_SIZE"] + pm["WRITE_SIZE"]) * 1024.0,
                      fetch_kb=pm["FETCH_SIZE"], write_kb=pm["WRITE_SIZE"])
        if "SQ_ACTIVE_INST_VALU" in pm and "GRBM_GUI_ACTIVE" in pm:
            # rocprof's VALUBusy (gfx9 formula: 4 x SQ_ACTIVE_INST_VALU / (SIMDs x GRBM_GUI_ACTIVE per XCD);
            # SQ_ACTIVE_INST_VALU is quad-cycles summed over resident waves)
            pj["valu_busy"] = 4.0 * pm["SQ_ACTIVE_INST_VALU"] / (1024.0 * pm["GRBM_GUI_ACTIVE"] / 8.0)
        if "SQ_WAVE_CYCLES" in pm and pm["SQ_WAVE_CYCLES"] > 0:
            pj["wave_cycles"] = {k[3:].lower(): pm[k] / pm["SQ_WAVE_CYCLES"] for k in
                                 ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if k in pm}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in pm and "GRBM_GUI_ACTIVE" in pm:
            pj["mfma_busy"] = pm["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * pm["GRBM_GUI_ACTIVE"] / 8.0)
        if "SQ_INSTS_VALU" in pm and "GRBM_GUI_ACTIVE" in pm:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs; a wave64 VALU op issues in 2 cycles
            cyc = pm["GRBM_GUI_ACTIVE"] / 8.0
            pj.update(valu_instr_per_simd_cycle=pm["SQ_INSTS_VALU"] / 1024.0 / cyc,
                      valu_issue_fraction=2.0 * pm["SQ_INSTS_VALU"] / 1024.0 / cyc,
                      gui_cycles_per_xcd=cyc,
                      effective_clock_ghz=cyc / res["timed_avg_ns"] if res.get("timed_avg_ns") else None)
        with open(a.pmc_json, "w") as f:
            json.dump(pj, f, indent=1)
    with open(a.out + ".json", "w") as f:
        json.dump(res, f, indent=1)
    with open(a.out + ".txt", "w") as f:
        f.write(f"rocprofv3 summary, {KERNEL}\n{a.note}\n")
        for k, v in res.items():
            if k != "stats_top":
                f.write(f"{k}: {v}\n")
        for s in res.get("stats_top", []):
            f.write(f"  {s['pct']:6.2f}%  {s['calls']:6d} calls  {s['avg_ns'] / 1e3:10.1f} us avg  {s['name']}\n")
    print(json.dumps({k: v for k, v in res.items() if k != "stats_top"}))


if __name__ == "__main__":
    main()
