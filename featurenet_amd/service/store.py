"""SQLite task store for the NAS service.

Schema is the reference's ``samples.db`` table (``tasks(id, timestamp, status,
params, task_id)``), so an existing database opens unchanged; all task fields
other than the id/status/timestamp live in the ``params`` JSON column.

Unlike the reference (``ui/back/main.py:55-143``: every forked process opens
the DB and writes whole rows, racing each other), updates here are
field-level JSON merges inside ``BEGIN IMMEDIATE`` transactions in WAL mode,
so the API process and any number of worker processes can update the same
task concurrently without lost writes.
"""
from __future__ import annotations

import json
import re
import sqlite3
import time
import uuid
from contextlib import contextmanager
from pathlib import Path

SCHEMA = """CREATE TABLE IF NOT EXISTS tasks (
    id INTEGER NOT NULL,
    timestamp FLOAT,
    status TEXT,
    params TEXT,
    task_id TEXT,
    PRIMARY KEY (id)
)"""


# fields only the server / worker may set: file locations that routes serve from
# and the worker writes to, and the task bookkeeping columns
SERVER_KEYS = frozenset({"products", "pdt", "fm", "fm_template", "error", "status", "task_id", "timestamp",
                         "valid_elements", "nb_valid_elements", "models"})


def safe_name(name) -> str:
    """A task name usable as ONE path component: [A-Za-z0-9_-], spaces -> '_' (reference
    ``ui/back/main.py`` replaced spaces only, so '../..' escaped the products directory)."""
    s = re.sub(r"[^A-Za-z0-9_-]", "", str(name).replace(" ", "_"))
    return s[:64]


class TaskStore:
    def __init__(self, path: str | Path):
        self.path = str(path)
        Path(self.path).parent.mkdir(parents=True, exist_ok=True)
        with self._conn() as c:
            c.execute(SCHEMA)
            c.execute("CREATE INDEX IF NOT EXISTS tasks_task_id ON tasks(task_id)")

    @contextmanager
    def _conn(self):
        c = sqlite3.connect(self.path, timeout=30, isolation_level=None)
        try:
            c.execute("PRAGMA journal_mode=WAL")
            c.execute("BEGIN IMMEDIATE")
            yield c
            c.execute("COMMIT")
        except BaseException:
            c.execute("ROLLBACK")
            raise
        finally:
            c.close()

    @staticmethod
    def _row(r) -> dict:
        if r is None:
            return None
        _, ts, status, params, task_id = r
        d = json.loads(params) if params else {}
        d.update({"task_id": task_id, "status": status, "timestamp": ts})
        return d

    def create(self, params: dict, status: str = "init") -> dict:
        # client data never sets server-owned fields (paths the worker writes or serves from)
        params = {k: v for k, v in dict(params or {}).items() if k not in SERVER_KEYS}
        params["task_name"] = safe_name(params.get("task_name", ""))
        task_id = uuid.uuid1().hex[:10]
        ts = int(time.time())
        with self._conn() as c:
            c.execute("INSERT INTO tasks(timestamp, status, params, task_id) VALUES (?,?,?,?)",
                      (ts, status, json.dumps(params), task_id))
        return {**params, "status": status, "timestamp": ts, "task_id": task_id}

    def get(self, task_id: str) -> dict | None:
        with self._conn() as c:
            return self._row(c.execute("SELECT id, timestamp, status, params, task_id FROM tasks WHERE task_id=?",
                                       (task_id,)).fetchone())

    def all(self) -> list[dict]:
        with self._conn() as c:
            rows = c.execute("SELECT id, timestamp, status, params, task_id FROM tasks ORDER BY id").fetchall()
        return [self._row(r) for r in rows]

    def update(self, task_id: str, status: str | None = None, **fields) -> dict | None:
        with self._conn() as c:
            r = c.execute("SELECT params FROM tasks WHERE task_id=?", (task_id,)).fetchone()
            if r is None:
                return None
            params = json.loads(r[0]) if r[0] else {}
            params.update(fields)
            if status is None:
                c.execute("UPDATE tasks SET params=? WHERE task_id=?", (json.dumps(params), task_id))
            else:
                c.execute("UPDATE tasks SET params=?, status=? WHERE task_id=?", (json.dumps(params), status, task_id))
        return self.get(task_id)

    def delete_all(self) -> int:
        with self._conn() as c:
            n = c.execute("SELECT COUNT(*) FROM tasks").fetchone()[0]
            c.execute("DELETE FROM tasks")
        return n
