"""SQ counters of the resident worker's dispatch (k_door) from rocprofv3
--pmc databases: totals and per read.  Usage:
    python3 scripts/sq_door_stats.py READS label=path/to/sq_results.db ..."""
import json
import sqlite3
import sys


def door_totals(db: str) -> dict:
    c = sqlite3.connect(db)
    rows = c.execute("SELECT counter_name, SUM(value) FROM counters_collection "
                     "WHERE kernel_name LIKE '%k_door%' GROUP BY counter_name")
    return {name: float(v) for name, v in rows}


reads = int(sys.argv[1])
out = {"reads": reads, "note": "SQ counters summed over k_door's dispatch(es) serving door_phases.py's reads "
       "(idle polling included); per_read = total / reads", "total": {}, "per_read": {}}
for arg in sys.argv[2:]:
    label, db = arg.split("=", 1)
    t = door_totals(db)
    out["total"][label] = t
    out["per_read"][label] = {k: round(v / reads, 1) for k, v in t.items()}
print(json.dumps(out, indent=1))
