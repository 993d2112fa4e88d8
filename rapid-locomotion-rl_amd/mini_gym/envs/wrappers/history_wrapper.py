from lrl.history import HistoryWrapper  # noqa: F401
