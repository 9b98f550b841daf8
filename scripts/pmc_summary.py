"""Summarise the rocprofv3 PMC passes of scripts/pmc.sh / pmc_cfg.sh for the fused kernel.

    python scripts/pmc_summary.py gpurun_out/pmc profiles/r01_c3_pmc.json [WORKLOAD ALG_BYTES KERNEL]

Per-launch means over the cm_predict_kernel dispatches of each pass.  HBM bytes follow the
MI355X guide's HBM/rocprofv3 section: FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
reports half the bytes of 16-B-per-lane streaming reads (the packed W stream is exactly that),
so it is doubled; WRITE_SIZE is exact for the 16-B stores of the epilogue.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = os.environ.get("PMC_KERNEL", "predict_kernel")   # cm_ (f64) and cm32_ (f32) fused kernels


def main(src, dst, workload="C3", alg_bytes=40 * 1048576, kernel_label="cm_predict_kernel<2, true, true>"):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(src, "p*", "*counter_collection.csv"))):
        with open(f) as fh:
            per_dispatch = defaultdict(dict)
            for row in csv.DictReader(fh):
                if KERNEL not in row["Kernel_Name"]:
                    continue
                d = per_dispatch[row["Dispatch_Id"]]
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            for d in per_dispatch.values():
                for k, v in d.items():
                    vals[k].append(v)
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    import hashlib
    lib = os.environ.get("BO_AMD_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "bayesopt_smart_amd", "libbo_amd.so"))
    with open(lib, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import device_code_sha256
    out = {"workload": workload, "kernel": kernel_label, "lib_sha256": lib_sha,
           "fatbin_sha256": device_code_sha256(lib),
           "counters_per_launch": mean, "launches_per_counter": {k: len(v) for k, v in vals.items()}}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        fetch = 2.0 * mean["FETCH_SIZE"] * 1024.0       # gfx950 16-B-read correction
        write = mean["WRITE_SIZE"] * 1024.0
        out.update({"fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                    "hbm_bytes_per_launch": fetch + write,
                    "note": "FETCH_SIZE x2 (gfx950 16-B streaming-read correction), KiB -> B; "
                            "algorithmic = outputs written (+ explicit coordinates read)"})
        if alg_bytes and alg_bytes > 1.0:   # no ratio without a real algorithmic byte count
            out.update({"algorithmic_bytes_per_launch": alg_bytes,
                        "traffic_ratio": (fetch + write) / alg_bytes})
        if os.environ.get("PMC_ALG_NOTE"):
            out["algorithmic_bytes_basis"] = os.environ["PMC_ALG_NOTE"]
    if "SQ_INSTS_MFMA" in mean and "SQ_INSTS_VALU" in mean:
        out["valu_per_mfma"] = mean["SQ_INSTS_VALU"] / max(mean["SQ_INSTS_MFMA"], 1.0)
        # SQ_INSTS_VALU counts the MFMAs too (C4: 2.7 per MFMA against ~1.7 other VALU per MFMA
        # counted in the ISA); the other vector ALU instructions per MFMA:
        out["non_mfma_valu_per_mfma"] = out["valu_per_mfma"] - 1.0
    if "SQ_WAIT_INST_ANY" in mean and "SQ_BUSY_CYCLES" in mean:
        out["wait_inst_any_per_busy_cycle"] = mean["SQ_WAIT_INST_ANY"] / max(mean["SQ_BUSY_CYCLES"], 1.0)
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], *([a[2], (None if a[3] == "none" else float(a[3]))] + a[4:5] if len(a) > 2 else []))
