"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs).

python scripts/pmc_traffic.py <fetch_dir> <write_dir> <n> <vlen> <kind> [<issue_dir>] > profiles/rNN/traffic.json

The output carries the library's source_id (pmc_codec.source_id()): bench.py quotes the traffic only
for the kernel sources it was measured on.  With <issue_dir> (a pass over SQ_INSTS_SALU SQ_INSTS_VALU
SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE) each kernel also gets "issue": the scalar unit's busy
fraction (SALU instructions per CU-cycle; one scalar unit per CU issues at most one per cycle), the
vector ALUs' (VALU instructions per SIMD-cycle, 4 SIMDs per CU) and the fraction of wave lifetime parked
on s_waitcnt.  CU-cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs) x 256 CUs.

FETCH_SIZE/WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md (HBM section) gfx950's FETCH_SIZE
counts half the bytes of wide coalesced reads; the correction (x2) is checked on this code's
own access pattern with compare_values_kernel, whose read bytes are known exactly
(2 * n * vlen + lengths): the reported 'fetch_calibration' is corrected/known and must be ~1.
"""
import csv
import json
import os
import sys


def per_kernel(d, counter):
    out = {}
    f = os.path.join(d, "run_counter_collection.csv")
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        out.setdefault(k, []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def issue(d):
    """per kernel: {counter: mean value per launch} from one pass."""
    out = {}
    f = os.path.join(d, "run_counter_collection.csv")
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        key = (r.get("Dispatch_Id") or r.get("Correlation_Id") or "")
        out.setdefault(k, {}).setdefault(r["Counter_Name"], {})
        c = out[k][r["Counter_Name"]]
        c[key] = c.get(key, 0.0) + float(r["Counter_Value"])
    res = {}
    for k, cs in out.items():
        m = {name: sum(v.values()) / len(v) for name, v in cs.items() if v}
        cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 * 256.0
        if not cyc:
            continue
        res[k] = {"salu_busy": m.get("SQ_INSTS_SALU", 0.0) / cyc,
                  "valu_busy": m.get("SQ_INSTS_VALU", 0.0) / (4.0 * cyc),
                  "wait_frac": m.get("SQ_WAIT_ANY", 0.0) / max(m.get("SQ_WAVE_CYCLES", 0.0), 1.0),
                  "counters_per_launch": m}
    return res


def main():
    fd, wd, n, vlen, kind = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    iss = issue(sys.argv[6]) if len(sys.argv) > 6 else {}
    fe, wr = per_kernel(fd, "FETCH_SIZE"), per_kernel(wd, "WRITE_SIZE")
    avg = lambda v: sum(v) / len(v) if v else None  # noqa: E731
    cal = None
    if "pmc::compare_values_kernel" in fe:
        known = 2.0 * n * vlen + 8.0 * n
        cal = 2.0 * avg(fe["pmc::compare_values_kernel"]) / known
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "poor-man-s-cache_amd"))
    import pmc_codec
    res = {"n": n, "vlen": vlen, "kind": kind, "source_id": pmc_codec.source_id(),
           "fetch_correction": 2.0, "fetch_calibration": cal,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, bench.py workload"}
    res["kernels"] = {}
    for k in sorted(set(fe) & set(wr)):
        if not k.startswith("pmc::"):
            continue
        f, w = avg(fe[k]), avg(wr[k])
        res["kernels"][k] = {"launches": len(fe[k]), "fetch_bytes_per_launch": 2.0 * f,
                             "write_bytes_per_launch": w, "hbm_bytes_per_launch": 2.0 * f + w}
        if k in iss:
            res["kernels"][k]["issue"] = iss[k]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
