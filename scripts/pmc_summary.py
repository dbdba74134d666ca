"""Per-kernel HBM traffic from two rocprofv3 PMC passes (scripts/gpu_profile.sh) -> a JSON summary.

    python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_v3_pmc.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. Correction (MI355X_MICROARCH.md, HBM section): on gfx950
FETCH_SIZE reports half of the bytes of a wide coalesced streaming read, so read bytes = 2 x FETCH_SIZE;
WRITE_SIZE is taken as reported. `eval_pass` sums the two kernels of one evaluation pass (eval_kernel and
eval_numa_kernel, one launch each per batch), which bench.py reports as roofline.traffic."""
import collections
import csv
import json
import os
import sys


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[name].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    f = per_kernel(fetch_dir, "FETCH_SIZE")
    w = per_kernel(write_dir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        fk = f.get(k, (0.0, 0))[0]
        wk = w.get(k, (0.0, 0))[0]
        kernels[k] = {"dispatches": max(f.get(k, (0, 0))[1], w.get(k, (0, 0))[1]),
                      "FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
                      "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024}
    ev = [k for k in kernels if k.startswith("gs::eval_") or k.startswith("gs::gather_numa")]
    res = {
        "note": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py --steps 1 "
                "--warmup 0 (C3); per-dispatch means; read bytes = 2 x FETCH_SIZE (gfx950 correction)",
        "kernels": kernels,
        "eval_pass": {"kernels": ev, "hbm_bytes_per_launch": sum(kernels[k]["hbm_bytes_per_launch"] for k in ev)},
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res["eval_pass"]))


if __name__ == "__main__":
    main()
