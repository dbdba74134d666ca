"""In-tree build of libgpuscore.so for gfx950 (hipcc; no JIT cache, the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libgpuscore.so")
SOURCES = ["gs_engine.cpp", "gs_numa_host.cpp", "gs_ingest.cpp", "gs_quota.cpp", "gs_reasons.cpp", "gs_kernels.hip", "gs_commit.hip", "gs_commit_spec.hip", "gs_probe.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fno-fast-math", "-Wall"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(HERE, "..", "include", "gpuscore.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC, *FLAGS, "-o", OUT + ".tmp", *[os.path.join(CSRC, s) for s in SOURCES], "-L/opt/rocm/lib", "-lrccl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
