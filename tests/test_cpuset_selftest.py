"""The bit-plane cpuset selection the commit kernel runs (koordinator_amd/csrc/gs_cpuset_dev.h) against the host
restatement of takeCPUs / allocateCPUSet (gs_numa_host.cpp, itself checked against the reference's
cpu_accumulator_test.go vectors in test_numa_golden.py and against the oracle on the GPU). Runs on the CPU: the
library compiles the same header for the host and exports a randomized self-test (no GPU call)."""
import ctypes as C

from koordinator_amd import abi


def run(seed, iters):
    lib = abi.load()
    fn = lib.gsx_cpuset_selftest
    fn.restype = C.c_int
    fn.argtypes = [C.c_uint64, C.c_int, C.c_char_p, C.c_size_t]
    buf = C.create_string_buffer(512)
    bad = fn(seed, iters, buf, len(buf))
    return bad, buf.value.decode()


def test_device_take_cpus_matches_host_restatement():
    bad, msg = run(0x6B6F6F7264, 20000)
    assert bad == 0, msg


def test_device_take_cpus_more_seeds():
    for seed in (1, 2, 3, 0xC0FFEE):
        bad, msg = run(seed, 4000)
        assert bad == 0, f"seed {seed}: {msg}"
