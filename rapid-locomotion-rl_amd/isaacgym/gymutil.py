"""``isaacgym.gymutil``: the device-string parser base_task.py:21 calls; the viewer helpers (draw_lines,
WireframeSphereGeometry) are out of scope (no viewer)."""


def parse_device_str(device_str):
    if device_str in ("cpu", "cuda"):
        return device_str, 0
    kind, _, idx = device_str.partition(":")
    return kind, int(idx or 0)


def parse_sim_config(cfg, sim_params):
    return sim_params
