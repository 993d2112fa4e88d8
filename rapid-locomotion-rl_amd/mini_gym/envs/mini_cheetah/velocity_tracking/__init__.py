from lrl.env import VelocityTrackingEasyEnv  # noqa: F401
