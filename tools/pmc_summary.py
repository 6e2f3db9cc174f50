"""Summarise the rocprofv3 counter passes of tools/profile_round.sh into profiles/pmc_traffic_<cfg>_b<B>.json.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950 FETCH_SIZE reports half the bytes of
16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM), and every weight load here is a 16 B/lane dwordx4;
WRITE_SIZE is exact for such stores.  MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x
1024 SIMDs)."""
import csv
import json
import statistics
import sys
from collections import defaultdict

prof, out = sys.argv[1], sys.argv[2]


def per_dispatch(path):
    agg = defaultdict(float)
    for r in csv.DictReader(open(path)):
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    res = defaultdict(list)
    for (d, c), v in sorted(agg.items()):
        res[c].append(v)
    return res


f = per_dispatch(f"{prof}/fetch/run_counter_collection.csv")["FETCH_SIZE"]
w = per_dispatch(f"{prof}/write/run_counter_collection.csv")["WRITE_SIZE"]
m = per_dispatch(f"{prof}/mfma/run_counter_collection.csv")
fetch_kib, write_kib = statistics.median(f), statistics.median(w)
busy = statistics.median(m["SQ_VALU_MFMA_BUSY_CYCLES"])
gui = statistics.median(m["GRBM_GUI_ACTIVE"])
res = {
    "kernel": "integrate_kernel<4,0,3,3> (LJ13, B=1024, Euler NFE=100)",
    "fetch_size_kib_raw": fetch_kib,
    "write_size_kib": write_kib,
    "hbm_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
    "note": "FETCH_SIZE doubled per the gfx950 16-B/lane correction; Infinity-Cache hits are counted in it",
    "sq_valu_mfma_busy_cycles": busy,
    "grbm_gui_active": gui,
    "mfma_pipe_busy_frac": busy / (gui / 8 * 1024),
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
