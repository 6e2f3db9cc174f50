"""Summarise tools/profile_configs.sh output: per case, the bench line (HIP-event ms per launch), the rocprofv3 kernel
trace average of integrate_kernel (per solve: a re-dealt adaptive solve is two launches), and the counter passes (HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE with the
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
        allstats = rows(os.path.join(d, "kt", "**", "*kernel_stats.csv"))
        stats = [r for r in allstats if "integrate_kernel" in r["Name"]]
        # a re-dealt adaptive solve (ecnf_hip.hip redeal_kernel) is two integrate launches: every per-launch figure
        # below is per SOLVE, summed over its launches
        # (the two launches may be different instantiations: the second one of an ALDP Hutchinson solve is the team
        # kernel with its tail teams; the per-solve time is the sum over every integrate row / the solves)
        # tools/profile_configs.sh runs each case as 1 warm-up + 2 timed solves (bench_paths --reps 2): the launches
        # per solve are the integrate launches / 3 (1; 2: re-dealt; 3: with ALDP's tail teams and stop-and-team)
        calls = sum(int(r["Calls"]) for r in stats)
        per = max(1, calls // 3)
        kt_avg_ms = sum(float(r["TotalDurationNs"]) for r in stats) * 1e-6 / (calls // per) if stats else None
        rec = {"case": case, "bench_ms": line["ms"], "tflops": line["tflops"], "nfe_mean": line["nfe_mean"],
               "rocprof_avg_ms": kt_avg_ms, "rocprof_calls": calls // per if stats else None,
               "launches_per_solve": per, "frac_of_split_peak": line["tflops"] / PEAK_SPLIT}
        c0, d0 = per_dispatch(os.path.join(d, "p0"))
        c1, _ = per_dispatch(os.path.join(d, "p1"))
        if c0 and c1:
            def solves(c, dd=None):
                ks = sorted(c)
                groups = [ks[i:i + per] for i in range(0, len(ks) - per + 1, per)]
                groups = groups[1:] or groups     # drop the warm-up solve
                return [({n: sum(c[k][n] for k in g) for n in c[g[0]]},
                         sum(dd[k] for k in g) if dd and all(k in dd for k in g) else None) for g in groups]
            s0, s1 = solves(c0, d0), solves(c1)
            fetch = statistics.median(v["FETCH_SIZE"] for v, _ in s0)
            gui = statistics.median(v["GRBM_GUI_ACTIVE"] for v, _ in s0)
            busy = statistics.median(v["SQ_VALU_MFMA_BUSY_CYCLES"] for v, _ in s0)
            write = statistics.median(v["WRITE_SIZE"] for v, _ in s1)
            durs = [t for _, t in s0 if t]
            dur = statistics.median(durs) if durs else None
            rec.update({"hbm_bytes_per_launch": (2 * fetch + write) * 1024, "fetch_size_kib_raw": fetch,
                        "write_size_kib": write, "grbm_gui_active": gui,
                        "clock_ghz_grbm": gui / 8 / (dur * 1e-9) / 1e9 if dur else None,
                        "mfma_pipe_busy_frac": busy / (gui / 8 * 1024)})
        out.append(rec)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
