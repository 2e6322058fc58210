"""Per-dispatch durations by predecessor from a rocprofv3 database (tools/gpu_launch_attr.sh): for every
kernel name, the median duration keyed by the kernel that ran right before it.
    python tools/launch_attr.py run_results.db"""
import re
import sqlite3
import statistics
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
rows = c.execute("""select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d
                    join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start""").fetchall()


def short(n):
    n = re.sub(r"^_ZN5vqhmm\d+", "", n)
    return re.sub(r"(E[A-Z].*|\.kd)$", "", n)[:24]


acc = defaultdict(list)
for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
    acc[(short(n1), short(n0))].append((e1 - s1) / 1e3)
for (k, prev), v in sorted(acc.items(), key=lambda kv: -len(kv[1])):
    if len(v) >= 5 and ("vq_" not in k and "vq_" not in prev):
        print(f"{k:26s} after {prev:26s} n={len(v):4d} median {statistics.median(v):7.2f} us  min {min(v):7.2f}")
