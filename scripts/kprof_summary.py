"""Per-kernel summary (calls, average / min duration) from rocprofv3 rocpd databases (*.db)."""
import sqlite3
import sys


def summary(db, top=30):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(duration), min(duration), sum(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    return rows[:top]


if __name__ == "__main__":
    for db in sys.argv[1:]:
        print(db)
        for name, n, avg, mn, tot in summary(db):
            print(f"  {name[:96]:96s} {n:5d} {avg / 1e3:8.2f} {mn / 1e3:8.2f} us")
