"""Commit-chain timeline from a rocprofv3 kernel trace: per batch, commit duration and the kernels / gaps between one
commit's end and the next commit's start (median over batches).

    python scripts/timeline.py gpurun_out/prof/bench_kernel_trace.csv
"""
import csv
import statistics
import sys


def main(path):
    ev = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    ev.sort()
    com = [e for e in ev if e[2].startswith("commit_spec")]
    print("commits", len(com))
    period = [(b[0] - a[0]) / 1e3 for a, b in zip(com, com[1:])]
    print("commit period us: median %.1f mean %.1f" % (statistics.median(period), statistics.mean(period)))
    print("commit duration us: median %.1f" % statistics.median([(c[1] - c[0]) / 1e3 for c in com]))
    # kernels fully between commit i's end and commit i+1's start, on the chain (started after commit i ended)
    between = {}
    gaps = []
    for a, b in zip(com, com[1:]):
        ks = [e for e in ev if e[0] >= a[1] and e[1] <= b[0]]
        gaps.append((b[0] - a[1]) / 1e3)
        for e in ks:
            between.setdefault(e[2], []).append(((e[0] - a[1]) / 1e3, (e[1] - e[0]) / 1e3))
    print("commit end -> next commit start us: median %.1f" % statistics.median(gaps))
    for n, v in sorted(between.items(), key=lambda kv: statistics.median([x[0] for x in kv[1]])):
        print("  %-28s n=%4d start +%.1f us dur %.1f us (median)" % (n, len(v), statistics.median([x[0] for x in v]),
                                                                  statistics.median([x[1] for x in v])))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/bench_kernel_trace.csv")
