"""Per-kernel duration summary from a rocprofv3 rocpd database (the default output
format of this rocprofv3): name, calls, total / average / min / max microseconds."""
import sqlite3
import sys


def main(path, top=30):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name}, count(*), sum(end-start), avg(end-start), min(end-start), "
                     f"max(end-start) from kernels group by {name} order by sum(end-start) desc "
                     f"limit {int(top)}").fetchall()
    print("calls,total_us,avg_us,min_us,max_us,name")
    for n, k, tot, avg, mn, mx in rows:
        print(f"{k},{tot / 1e3:.1f},{avg / 1e3:.2f},{mn / 1e3:.2f},{mx / 1e3:.2f},{n[:150]}")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []))
