#!/usr/bin/env python
"""Close a kernel's wave cycles from SQ counters.

    python tools/pmc_close.py <pass dir>...      (rocprofv3 --pmc output directories)

Averages each counter over the dispatches of the passes (one kernel regex per run) and prints the
decomposition WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY vs WAVE_CYCLES (all quad-cycles, summed
over waves; MI355X_MICROARCH.md PMC table), per-SIMD busy fractions of the VALU / LDS / matrix
pipes over the dispatch's clock (GRBM_GUI_ACTIVE / 8 XCDs), and instruction mixes per wave.
"""
import collections
import csv
import glob
import json
import sys


def load(dirs):
    acc = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    m = load(sys.argv[1:])
    print(" ".join(f"{k}={v:.4g}" for k, v in sorted(m.items())))
    simds = 1024
    clk = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0  # cycles of the dispatch (GRBM sums the 8 XCDs)
    wc = m.get("SQ_WAVE_CYCLES", 0.0)
    out = {"dispatch_cycles": clk}
    if wc:
        parts = {k: m.get(k, 0.0) / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
        parts["sum"] = sum(parts.values())
        parts["SQ_WAIT_INST_LDS (part of WAIT_INST_ANY)"] = m.get("SQ_WAIT_INST_LDS", 0.0) / wc
        for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC",
                  "SQ_ACTIVE_INST_FLAT", "SQ_INST_CYCLES_VMEM"):
            if k in m:
                parts[k] = m[k] / wc
        out["of_wave_cycles"] = parts
        out["waves_per_simd"] = 4.0 * wc / (clk * simds) if clk else None
    if clk:
        busy = {}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            busy["mfma_busy_per_simd"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * simds)
        if "SQ_LDS_IDX_ACTIVE" in m:
            busy["lds_array_busy_per_cu"] = m["SQ_LDS_IDX_ACTIVE"] / (clk * 256)
        if "SQ_ACTIVE_INST_VALU" in m:
            busy["active_inst_valu_per_simd (4 x quad-cycles)"] = 4 * m["SQ_ACTIVE_INST_VALU"] / (clk * simds)
        if "SQ_INSTS_VALU" in m:
            busy["valu_winstr_per_simd_cycle"] = m["SQ_INSTS_VALU"] / (clk * simds)
        if "SQ_INSTS_LDS" in m:
            busy["lds_winstr_per_cu_cycle"] = m["SQ_INSTS_LDS"] / (clk * 256)
        out["busy"] = busy
    if "SQ_WAVES" in m:
        w = m["SQ_WAVES"]
        out["per_wave"] = {k: m[k] / w for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM",
                                                 "SQ_INSTS_MFMA", "SQ_INSTS_SMEM") if k in m}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
