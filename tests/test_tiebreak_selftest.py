"""selectHost's tie-break position as the speculative commit kernel computes it: per-pod reservoir records built in
the kernel's prologue (tiebreak_records, gs_eval_dev.h) and a lane-parallel count over them (gs_commit_spec.hip
tb_pos), against the reservoir walk itself (tiebreak_position, the host oracle's tie-break). Runs on the CPU: the
library compiles the same header for the host and exports a randomized self-test (no GPU call)."""
import ctypes as C

from koordinator_amd import abi


def run(seed, iters):
    lib = abi.load()
    fn = lib.gsx_tiebreak_selftest
    fn.restype = C.c_int
    fn.argtypes = [C.c_uint64, C.c_int, C.c_char_p, C.c_size_t]
    buf = C.create_string_buffer(512)
    bad = fn(seed, iters, buf, len(buf))
    return bad, buf.value.decode()


def test_tiebreak_records_lookup_matches_walk():
    bad, msg = run(0x6B6F6F7264, 20000)
    assert bad == 0, msg


def test_tiebreak_records_more_seeds():
    for seed in (1, 2, 0xC0FFEE):
        bad, msg = run(seed, 3000)
        assert bad == 0, f"seed {seed}: {msg}"
