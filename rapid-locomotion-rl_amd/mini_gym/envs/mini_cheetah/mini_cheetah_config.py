from lrl.config import config_mini_cheetah  # noqa: F401
