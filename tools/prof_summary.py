"""Per-kernel summary of a rocprofv3 SQLite trace (results.db): calls, avg and total time."""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(duration), sum(duration) from kernels "
                     "group by name order by sum(duration) desc").fetchall()
    tot = sum(r[3] for r in rows)
    print(f"{'kernel':<80} {'calls':>6} {'avg_us':>10} {'total_ms':>10} {'%':>6}")
    for name, n, avg, s in rows[:top]:
        print(f"{name[:80]:<80} {n:>6} {avg / 1e3:>10.2f} {s / 1e6:>10.3f} {100 * s / tot:>6.2f}")


if __name__ == "__main__":
    main()
