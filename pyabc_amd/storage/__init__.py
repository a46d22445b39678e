from .history import History, create_sqlite_db_id
