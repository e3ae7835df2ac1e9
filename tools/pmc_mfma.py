#!/usr/bin/env python3
"""MFMA utilisation per kernel kind from one rocprofv3 --pmc pass (tools/round_end.sh):
SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F32 / _BF16, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES,
GRBM_GUI_ACTIVE, with --kernel-trace in the same run for the dispatch durations.

Units (MI355X_MICROARCH.md:42, :488): one MOPS unit is 512 FLOPs; SQ_VALU_MFMA_BUSY_CYCLES counts
SIMD cycles summed over the chip (for v_mfma_f32_16x16x4_f32 it reads exactly 8 x MOPS_F32: 2048
FLOPs per instruction at 64 FLOP/clk/SIMD = 32 cycles).  MFMA utilisation of a launch = busy cycles
/ (duration x 2.4 GHz x 256 CUs x 4 SIMDs); GRBM_GUI_ACTIVE is the sum over the 8 XCDs and reads
high on dispatches this short (the guide's DVFS note), so the kernel trace's duration is the
denominator.  Traced durations carry the profiler's per-dispatch overhead; bench.py divides the
counter figures by its own live launch time instead.

usage: pmc_mfma.py OUT_JSON WORKLOAD=DIR [WORKLOAD=DIR ...]"""
import collections
import csv
import json
import os
import sys

CLK_HZ = 2.4e9
SIMDS = 256 * 4
FP32_PEAK = 157.3e12   # MI355X_MICROARCH.md:42 (matrix fp32, dense)
BF16_PEAK = 2.5e15     # MI355X_MICROARCH.md:43 (dense)
KINDS = ("k_bwd", "k_fwd", "k_ver", "k_tdg", "k_gpi", "k_sel1m", "k_qmax", "k_tsf")


def kind_of(name):
    base = name.split("(")[0].split("<")[0].split("::")[-1].strip()
    for k in KINDS:
        if base == k or base.startswith(k + "_"):
            return "k_bwd" if base.startswith("k_bwd") else k
    return None


def summarise(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = kind_of(r["Kernel_Name"])
        if k:
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    dur = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        k = kind_of(r["Kernel_Name"])
        if k:
            dur[k][0] += 1
            dur[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k, c in per.items():
        n = len(disp[k])
        busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / n
        f32 = c["SQ_INSTS_VALU_MFMA_MOPS_F32"] * 512.0 / n
        bf16 = c["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512.0 / n
        t = dur[k][1] / dur[k][0] if dur[k][0] else None
        out[k] = {"launches": n, "mfma_busy_cycles_per_launch": round(busy),
                  "mfma_flops_f32_per_launch": round(f32), "mfma_flops_bf16_per_launch": round(bf16),
                  "sq_busy_cycles_per_launch": round(c["SQ_BUSY_CYCLES"] / n),
                  "sq_wave_cycles_per_launch": round(c["SQ_WAVE_CYCLES"] / n),
                  "grbm_gui_active_per_launch": round(c["GRBM_GUI_ACTIVE"] / n),
                  "traced_avg_us": None if t is None else round(t * 1e6, 3)}
        if t:
            out[k]["mfma_util_traced"] = round(busy / (t * CLK_HZ * SIMDS), 5)
            out[k]["compute_frac_traced"] = round(f32 / t / FP32_PEAK + bf16 / t / BF16_PEAK, 5)
    return out


def main(out_json, *pairs):
    rec = json.load(open(out_json)) if os.path.exists(out_json) else {}
    for p in pairs:
        wl, d = p.split("=", 1)
        rec[wl] = summarise(d)
        rec[wl]["_source"] = (f"rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 "
                              f"SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE "
                              f"--kernel-trace ({os.path.basename(d.rstrip('/'))}); tools/pmc_mfma.py")
    rec["_units"] = {"clock_hz": CLK_HZ, "simds": SIMDS, "fp32_mfma_peak_flops": FP32_PEAK,
                     "bf16_mfma_peak_flops": BF16_PEAK, "mops_unit_flops": 512,
                     "mfma_util": "busy cycles / (duration x clock x SIMDs)"}
    json.dump(rec, open(out_json, "w"), indent=1, sort_keys=True)
    print(json.dumps(rec, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(*sys.argv[1:])
