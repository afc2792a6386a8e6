"""Load health.csv into the SQL database the JDBC workloads read
(reference: infra/local/mysql-database/load_csv.py:21-174).

Same schema (``id`` auto-increment primary key, the 10 CSV columns with FLOAT measures,
``created_at`` default timestamp), NaN -> NULL, batched ``executemany`` of 1000 rows with a commit per
batch.  The database is SQLite (stdlib) at ``$PTG_JDBC_ROOT/<database>.sqlite`` — the file a
``jdbc:mysql://host:port/<database>`` URL resolves to in this runtime.

    python workloads/raw-spark/load_csv.py --csv tests/data/health.csv --root /tmp/db
"""
import argparse
import logging
import math
import os
import sqlite3

import pandas as pd

logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
logger = logging.getLogger("load_csv")

DB_CONFIG = {"database": "health_data", "table": "health_disparities"}
COLUMNS = ["edition", "report_type", "measure_name", "state_name", "subpopulation", "value", "lower_ci", "upper_ci",
           "source", "source_date"]
SCHEMA = """
CREATE TABLE IF NOT EXISTS health_disparities (
    id INTEGER PRIMARY KEY AUTOINCREMENT,
    edition VARCHAR(10),
    report_type VARCHAR(100),
    measure_name VARCHAR(100),
    state_name VARCHAR(50),
    subpopulation VARCHAR(100),
    value FLOAT,
    lower_ci FLOAT,
    upper_ci FLOAT,
    source VARCHAR(255),
    source_date VARCHAR(50),
    created_at TIMESTAMP DEFAULT CURRENT_TIMESTAMP
)
"""


def _clean(v):
    if v is None or (isinstance(v, float) and math.isnan(v)):
        return None
    return v.item() if hasattr(v, "item") else v


def load(csv_path: str, root: str, batch_size: int = 1000, truncate: bool = False) -> int:
    os.makedirs(root, exist_ok=True)
    db_path = os.path.join(root, f"{DB_CONFIG['database']}.sqlite")
    df = pd.read_csv(csv_path)
    logger.info(f"Read {len(df)} rows from {csv_path}")
    con = sqlite3.connect(db_path)
    try:
        con.execute(SCHEMA)
        logger.info("Table 'health_disparities' created or already exists.")
        if truncate:
            con.execute("DELETE FROM health_disparities")
            con.execute("DELETE FROM sqlite_sequence WHERE name = 'health_disparities'")
        cols = [c for c in COLUMNS if c in df.columns]
        q = f"INSERT INTO health_disparities ({', '.join(cols)}) VALUES ({', '.join('?' * len(cols))})"
        rows = [tuple(_clean(v) for v in r) for r in df[cols].itertuples(index=False)]
        inserted = 0
        for i in range(0, len(rows), batch_size):
            con.executemany(q, rows[i:i + batch_size])
            con.commit()
            inserted += len(rows[i:i + batch_size])
            logger.info(f"Inserted batch {i // batch_size + 1}: {inserted}/{len(rows)} rows")
    finally:
        con.close()
    logger.info(f"Database written to {db_path}")
    return inserted


def main(argv=None):
    here = os.path.dirname(os.path.abspath(__file__))
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--csv", default=os.environ.get("CSV_PATH", os.path.join(here, "..", "..", "tests", "data",
                                                                            "health.csv")))
    ap.add_argument("--root", default=os.environ.get("PTG_JDBC_ROOT", os.path.join(here, "db")))
    ap.add_argument("--batch-size", type=int, default=1000)
    ap.add_argument("--truncate", action="store_true", help="empty the table first (manege.sql)")
    a = ap.parse_args(argv)
    load(a.csv, a.root, a.batch_size, a.truncate)


if __name__ == "__main__":
    main()
