"""NAS task service: SQLite task store, REST API (FastAPI) and worker processes."""
