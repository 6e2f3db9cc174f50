"""Summarise tools/profile_configs.sh output: per case, the bench line (HIP-event ms per launch), the rocprofv3 kernel
trace average of integrate_kernel, and the counter passes (HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE with the
gfx950 16-B/lane FETCH_SIZE correction, effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration, MFMA pipe busy =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)).  Usage: python tools/pmc_configs.py PROFILE_DIR"""
import csv
import glob
import json
import os
import statistics
import sys

PEAK_SPLIT = 2516.6 / 3      # TFLOP/s: dense 16-bit MFMA peak / 3 split terms (bench.roofline_peak without the VALU share)


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        out += list(csv.DictReader(open(p)))
    return out


def per_dispatch(d):
    agg = {}
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        k = int(r["Dispatch_Id"])
        agg.setdefault(k, {})
        agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    durs = {int(r["Dispatch_Id"]): float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            for r in rows(os.path.join(d, "**", "*kernel_trace.csv")) if "integrate_kernel" in r["Kernel_Name"]}
    return agg, durs


def main(prof):
    out = []
    for d in sorted(glob.glob(os.path.join(prof, "*", ""))):
        case = os.path.basename(os.path.dirname(d))
        try:
            line = json.loads(open(os.path.join(d, "line_kt.json")).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        stats = [r for r in rows(os.path.join(d, "kt", "**", "*kernel_stats.csv")) if "integrate_kernel" in r["Name"]]
        kt_avg_ms = float(stats[0]["AverageNs"]) * 1e-6 if stats else None
        rec = {"case": case, "bench_ms": line["ms"], "tflops": line["tflops"], "nfe_mean": line["nfe_mean"],
               "rocprof_avg_ms": kt_avg_ms, "rocprof_calls": int(stats[0]["Calls"]) if stats else None,
               "frac_of_split_peak": line["tflops"] / PEAK_SPLIT}
        c0, d0 = per_dispatch(os.path.join(d, "p0"))
        c1, _ = per_dispatch(os.path.join(d, "p1"))
        if c0 and c1:
            k0 = sorted(c0)[1:] or sorted(c0)     # drop the warm-up dispatch
            k1 = sorted(c1)[1:] or sorted(c1)
            fetch = statistics.median(c0[k]["FETCH_SIZE"] for k in k0)
            gui = statistics.median(c0[k]["GRBM_GUI_ACTIVE"] for k in k0)
            busy = statistics.median(c0[k]["SQ_VALU_MFMA_BUSY_CYCLES"] for k in k0)
            write = statistics.median(c1[k]["WRITE_SIZE"] for k in k1)
            dur = statistics.median(d0[k] for k in k0 if k in d0) if d0 else None
            rec.update({"hbm_bytes_per_launch": (2 * fetch + write) * 1024, "fetch_size_kib_raw": fetch,
                        "write_size_kib": write, "grbm_gui_active": gui,
                        "clock_ghz_grbm": gui / 8 / (dur * 1e-9) / 1e9 if dur else None,
                        "mfma_pipe_busy_frac": busy / (gui / 8 * 1024)})
        out.append(rec)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
