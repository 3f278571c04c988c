"""Per-kernel PMC summary from tools/gpu_traffic.sh output -> JSON (bytes per launch).

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a wide (16 B/lane)
coalesced read, so it is doubled; WRITE_SIZE is exact for 16-B streaming stores.  The raw
TCC_EA0_RDREQ/WRREQ sums of the third pass are kept beside them for the unit check.
usage: traffic_table.py <traffic dir> <out.json>
"""
import collections, csv, glob, json, os, sys

root, out = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[(n, r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = {}
for (n, grid), d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    row = {"launches": max(len(v) for v in d.values())}
    if "FETCH_SIZE" in m:
        row["fetch_bytes_corrected"] = 2 * m["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in m:
        row["write_bytes"] = m["WRITE_SIZE"] * 1024
    for k in ("TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE",
              "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
        if k in m:
            row[k] = m[k]
    if "fetch_bytes_corrected" in row and "write_bytes" in row:
        row["hbm_bytes"] = row["fetch_bytes_corrected"] + row["write_bytes"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in row and row.get("GRBM_GUI_ACTIVE"):
        # MFMA busy = busy cycles / (wall cycles x 1024 SIMDs); GRBM_GUI_ACTIVE sums the 8 XCDs
        row["mfma_busy"] = row["SQ_VALU_MFMA_BUSY_CYCLES"] / (row["GRBM_GUI_ACTIVE"] / 8 * 1024)
    rows[f"{n} grid={grid}"] = row
json.dump(rows, open(out, "w"), indent=1, sort_keys=True)
for k, r in sorted(rows.items(), key=lambda kv: -kv[1].get("hbm_bytes", 0)):
    if "at::native" in k or "rocclr" in k:
        continue
    print(f"{k[:70]:70s} hbm={r.get('hbm_bytes', 0) / 1e6:10.1f} MB  mfma_busy={r.get('mfma_busy', 0):.3f} gui={r.get('GRBM_GUI_ACTIVE', 0):.3g}")
