"""Kernel stats (name, calls, total/avg/min/max ns) from a rocprofv3 rocpd sqlite database,
like the --stats kernel_stats.csv.  usage: python tools/rocpd_stats.py run_results.db [--csv out.csv]"""
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("""select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start),
                           min(d.end - d.start), max(d.end - d.start)
                    from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
                    group by s.kernel_name order by sum(d.end - d.start) desc""").fetchall()
tot = sum(r[2] for r in rows)
lines = ['"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"']
for n, k, t, a, mn, mx in rows:
    lines.append(f'"{n}",{k},{t},{a:.1f},{100.0 * t / tot:.2f},{mn},{mx}')
out = "\n".join(lines)
if "--csv" in sys.argv:
    open(sys.argv[sys.argv.index("--csv") + 1], "w").write(out + "\n")
for ln in lines[:40]:
    print(ln[:160])
