"""In-tree build of libgpuscore.so for gfx950 (hipcc; no JIT cache, the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libgpuscore.so")
SOURCES = ["gs_engine.cpp", "gs_numa_host.cpp", "gs_ingest.cpp", "gs_quota.cpp", "gs_gang.cpp", "gs_reasons.cpp",
           "gs_kernels.hip",
           "gs_commit_spec.hip", "gs_probe.hip", "gs_ext.hip"]
OBJ = os.path.join(HERE, "build")
# host code off the per-pod path whose -O3 build takes minutes in clang (the inlined cpuset selection of the
# self-test): -O2 (27 s instead of ~210 s)
O2_SOURCES = {"gs_numa_host.cpp"}
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fno-fast-math", "-Wall"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(HERE, "..", "include", "gpuscore.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def _objects(force: bool, verbose: bool) -> list[str]:
    """One object per source, compiled in parallel; a source is recompiled when it, or a header it includes (the
    compiler's dependency file), is newer than its object."""
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(OBJ, exist_ok=True)
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hdrs.append(os.path.join(HERE, "..", "include", "gpuscore.h"))
    newest_hdr = max(os.path.getmtime(h) for h in hdrs)

    def newest_dep(sp: str, dp: str) -> float:
        if not os.path.exists(dp):
            return max(os.path.getmtime(sp), newest_hdr)
        deps = open(dp).read().replace("\\\n", " ").split(":", 1)[-1].split()
        return max([os.path.getmtime(sp)] + [os.path.getmtime(d) if os.path.exists(d) else float("inf") for d in deps])

    jobs, objs = [], []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        op = os.path.join(OBJ, src + ".o")
        dp = op + ".d"
        objs.append(op)
        if force or not os.path.exists(op) or os.path.getmtime(op) < newest_dep(sp, dp):
            flags = [f for f in FLAGS if f != "-shared"]
            if src in O2_SOURCES:
                flags = ["-O2" if f == "-O3" else f for f in flags]
            jobs.append([HIPCC, *flags, "-MD", "-MF", dp, "-c", "-o", op + ".tmp", sp])
    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        os.replace(cmd[cmd.index("-o") + 1], cmd[cmd.index("-o") + 1][:-4])
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "8"))))
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(run, jobs))
    return objs


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    objs = _objects(force, verbose)
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp", *objs, "-L/opt/rocm/lib", "-lrccl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
