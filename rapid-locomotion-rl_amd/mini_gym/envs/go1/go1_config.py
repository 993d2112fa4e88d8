from lrl.config import config_go1  # noqa: F401
