from .history import History, create_sqlite_db_id
from .json import save_dict_to_json, load_dict_from_json
