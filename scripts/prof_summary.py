"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) per kernel symbol and grid:
count, total / avg / min / max duration (us), VGPRs, scratch. Usage:
    python scripts/prof_summary.py gpurun_out/prof/run_results.db [--by-symbol] [--top N]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--by-symbol", action="store_true", help="aggregate over grids")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    grp = "name" if a.by_symbol else "name, grid_x, grid_y, grid_z"
    q = (f"select name, count(*), sum(duration)/1e3, avg(duration)/1e3, min(duration)/1e3, "
         f"max(duration)/1e3, grid_x, grid_y, grid_z, max(vgpr_count), max(accum_vgpr_count), "
         f"max(scratch_size) from kernels group by {grp} order by sum(duration) desc limit {a.top}")
    tot = c.execute("select sum(duration)/1e3, count(*) from kernels").fetchone()
    print(f"# total kernel time {tot[0]:.1f} us over {tot[1]} dispatches")
    print(f"{'count':>6} {'total_us':>10} {'avg_us':>9} {'min_us':>9} {'max_us':>9} {'grid':>18} vgpr agpr scr  kernel")
    for r in c.execute(q):
        grid = f"{r[6]}x{r[7]}x{r[8]}" if not a.by_symbol else "-"
        print(f"{r[1]:6d} {r[2]:10.1f} {r[3]:9.2f} {r[4]:9.2f} {r[5]:9.2f} {grid:>18} {r[9]:4} {r[10]:4} {r[11]:3}  {r[0][:120]}")


if __name__ == "__main__":
    main()
