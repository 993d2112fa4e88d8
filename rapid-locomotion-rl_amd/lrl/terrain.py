"""Rough-terrain generation: the reference's ``Terrain`` (mini_gym/utils/terrain.py:
12-184) over a restatement of the Isaac Gym Preview ``terrain_utils`` primitives it calls.

``isaacgym.terrain_utils`` is not vendored in the reference and is not installable here, so the primitives
below follow its published algorithm (int16 height fields in units of ``vertical_scale``, sub-terrains of
``width x length`` pixels of ``horizontal_scale`` metres; the same ``np.random`` draw order) — parity
unpinned for the primitives themselves.  The layout logic on top (curriculum / randomized / selected tiles,
border, env origins) is pinned against the reference's own ``Terrain`` class driven by these primitives
(tests/golden/terrain.npz, tests/golden/make_golden.py).

The device side uses ``heights_m`` (metres, float32, [tot_rows, tot_cols], x = row * horizontal_scale -
border) for the contact ground height and the height scan (legged_robot.py:1469-1503).
"""
import numpy as np
from scipy.interpolate import RegularGridInterpolator


class SubTerrain:
    """One tile: ``height_field_raw`` int16 [width, length] in units of ``vertical_scale``."""

    def __init__(self, terrain_name="terrain", width=256, length=256, vertical_scale=1.0, horizontal_scale=1.0):
        self.terrain_name = terrain_name
        self.vertical_scale = vertical_scale
        self.horizontal_scale = horizontal_scale
        self.width = width
        self.length = length
        self.height_field_raw = np.zeros((width, length), dtype=np.int16)


def random_uniform_terrain(terrain, min_height, max_height, step=1, downsampled_scale=None):
    """Add uniform noise drawn on a coarse grid (every ``downsampled_scale`` metres) and bilinearly
    upsampled to the tile, rounded to whole vertical units."""
    vs, hs = terrain.vertical_scale, terrain.horizontal_scale
    if downsampled_scale is None:
        downsampled_scale = hs
    lo, hi, st = int(min_height / vs), int(max_height / vs), int(step / vs)
    levels = np.arange(lo, hi + st, st)
    nx = int(terrain.width * hs / downsampled_scale)
    ny = int(terrain.length * hs / downsampled_scale)
    coarse = np.random.choice(levels, (nx, ny))
    gx = np.linspace(0, terrain.width * hs, nx)
    gy = np.linspace(0, terrain.length * hs, ny)
    interp = RegularGridInterpolator((gx, gy), coarse.astype(np.float64), method="linear")
    fx = np.linspace(0, terrain.width * hs, terrain.width)
    fy = np.linspace(0, terrain.length * hs, terrain.length)
    X, Y = np.meshgrid(fx, fy, indexing="ij")
    fine = np.rint(interp(np.stack([X.ravel(), Y.ravel()], -1)).reshape(terrain.width, terrain.length))
    terrain.height_field_raw += fine.astype(np.int16)
    return terrain


def pyramid_sloped_terrain(terrain, slope=1, platform_size=1.0):
    """A four-sided pyramid (slope > 0) or pit (slope < 0) of the given slope, flattened to the height of
    the central platform's corner."""
    w, l = terrain.width, terrain.length
    cx, cy = int(w / 2), int(l / 2)
    fx = ((cx - np.abs(cx - np.arange(w))) / cx).reshape(w, 1)
    fy = ((cy - np.abs(cy - np.arange(l))) / cy).reshape(1, l)
    peak = int(slope * (terrain.horizontal_scale / terrain.vertical_scale) * (w / 2))
    terrain.height_field_raw += (peak * fx * fy).astype(terrain.height_field_raw.dtype)
    half = int(platform_size / terrain.horizontal_scale / 2)
    corner = terrain.height_field_raw[w // 2 - half, l // 2 - half]
    terrain.height_field_raw = np.clip(terrain.height_field_raw, min(corner, 0), max(corner, 0))
    return terrain


def pyramid_stairs_terrain(terrain, step_width, step_height, platform_size=1.0):
    """Concentric square steps rising (or, with step_height < 0, falling) towards a central platform."""
    sw = int(step_width / terrain.horizontal_scale)
    sh = int(step_height / terrain.vertical_scale)
    ps = int(platform_size / terrain.horizontal_scale)
    x0, x1, y0, y1, h = 0, terrain.width, 0, terrain.length, 0
    while (x1 - x0) > ps and (y1 - y0) > ps:
        x0, x1, y0, y1, h = x0 + sw, x1 - sw, y0 + sw, y1 - sw, h + sh
        terrain.height_field_raw[x0:x1, y0:y1] = h
    return terrain


def discrete_obstacles_terrain(terrain, max_height, min_size, max_size, num_rects, platform_size=1.0):
    """``num_rects`` random rectangular blocks at +-max_height or +-max_height/2, a flat central platform."""
    mh = int(max_height / terrain.vertical_scale)
    smin, smax = int(min_size / terrain.horizontal_scale), int(max_size / terrain.horizontal_scale)
    ps = int(platform_size / terrain.horizontal_scale)
    rows, cols = terrain.height_field_raw.shape
    heights = [-mh, -mh // 2, mh // 2, mh]
    sizes = range(smin, smax, 4)
    for _ in range(num_rects):
        w = np.random.choice(sizes)
        l = np.random.choice(sizes)
        i0 = np.random.choice(range(0, rows - w, 4))
        j0 = np.random.choice(range(0, cols - l, 4))
        terrain.height_field_raw[i0:i0 + w, j0:j0 + l] = np.random.choice(heights)
    x0, x1 = (terrain.width - ps) // 2, (terrain.width + ps) // 2
    y0, y1 = (terrain.length - ps) // 2, (terrain.length + ps) // 2
    terrain.height_field_raw[x0:x1, y0:y1] = 0
    return terrain


def stepping_stones_terrain(terrain, stone_size, stone_distance, max_height, platform_size=1.0, depth=-10):
    """Square stones separated by gaps ``depth`` metres deep, rows of stones along the longer side."""
    ss = int(stone_size / terrain.horizontal_scale)
    sd = int(stone_distance / terrain.horizontal_scale)
    mh = int(max_height / terrain.vertical_scale)
    ps = int(platform_size / terrain.horizontal_scale)
    levels = np.arange(-mh - 1, mh, step=1)
    hf = terrain.height_field_raw
    hf[:, :] = int(depth / terrain.vertical_scale)
    if terrain.length >= terrain.width:
        y = 0
        while y < terrain.length:
            y_end = min(terrain.length, y + ss)
            x = np.random.randint(0, ss)
            hf[0:max(0, x - sd), y:y_end] = np.random.choice(levels)  # the partial stone before the first
            while x < terrain.width:
                hf[x:min(terrain.width, x + ss), y:y_end] = np.random.choice(levels)
                x += ss + sd
            y += ss + sd
    else:
        x = 0
        while x < terrain.width:
            x_end = min(terrain.width, x + ss)
            y = np.random.randint(0, ss)
            hf[x:x_end, 0:max(0, y - sd)] = np.random.choice(levels)
            while y < terrain.length:
                hf[x:x_end, y:min(terrain.length, y + ss)] = np.random.choice(levels)
                y += ss + sd
            x += ss + sd
    x0, x1 = (terrain.width - ps) // 2, (terrain.width + ps) // 2
    y0, y1 = (terrain.length - ps) // 2, (terrain.length + ps) // 2
    hf[x0:x1, y0:y1] = 0
    return terrain


def convert_heightfield_to_trimesh(height_field_raw, horizontal_scale, vertical_scale, slope_threshold=None):
    """Vertices [rows*cols, 3] and triangles [2 (rows-1)(cols-1), 3] of the height field; with a slope
    threshold, vertices at the foot of a too-steep rise move one cell towards it (vertical walls)."""
    hf = height_field_raw.astype(np.int64)
    rows, cols = hf.shape
    xx, yy = np.meshgrid(np.linspace(0, (rows - 1) * horizontal_scale, rows),
                         np.linspace(0, (cols - 1) * horizontal_scale, cols), indexing="ij")
    if slope_threshold is not None:
        thr = slope_threshold * horizontal_scale / vertical_scale
        mx, my, mc = np.zeros((rows, cols)), np.zeros((rows, cols)), np.zeros((rows, cols))
        mx[:-1, :] += hf[1:, :] - hf[:-1, :] > thr
        mx[1:, :] -= hf[:-1, :] - hf[1:, :] > thr
        my[:, :-1] += hf[:, 1:] - hf[:, :-1] > thr
        my[:, 1:] -= hf[:, :-1] - hf[:, 1:] > thr
        mc[:-1, :-1] += hf[1:, 1:] - hf[:-1, :-1] > thr
        mc[1:, 1:] -= hf[:-1, :-1] - hf[1:, 1:] > thr
        xx = xx + (mx + mc * (mx == 0)) * horizontal_scale
        yy = yy + (my + mc * (my == 0)) * horizontal_scale
    vertices = np.stack([xx.ravel(), yy.ravel(), hf.ravel() * vertical_scale], -1).astype(np.float32)
    i0 = (np.arange(rows - 1)[:, None] * cols + np.arange(cols - 1)[None, :]).ravel()
    tri = np.empty((2 * (rows - 1) * (cols - 1), 3), dtype=np.uint32)
    tri[0::2] = np.stack([i0, i0 + cols + 1, i0 + 1], -1)
    tri[1::2] = np.stack([i0, i0 + cols, i0 + cols + 1], -1)
    return vertices, tri


class Terrain:
    """terrain.py:12-184: the tiled height field of ``num_rows`` difficulty levels x ``num_cols`` terrain
    types (curriculum), random tiles, or one selected type; ``env_origins`` [rows, cols, 3] per tile."""

    def __init__(self, cfg, num_robots, eval_cfg=None, num_eval_robots=0):
        self.cfg, self.eval_cfg, self.num_robots = cfg, eval_cfg, num_robots
        self.type = cfg.mesh_type
        if self.type in ("none", "plane"):
            return
        self.train_rows, self.train_cols, self.eval_rows, self.eval_cols = self._layout()
        self.tot_rows = len(self.train_rows) + len(self.eval_rows)
        self.tot_cols = max(len(self.train_cols), len(self.eval_cols))
        cfg.env_length, cfg.env_width = cfg.terrain_length, cfg.terrain_width
        self.height_field_raw = np.zeros((self.tot_rows, self.tot_cols), dtype=np.int16)
        for c in (cfg, eval_cfg):
            if c is None:
                continue
            if c.curriculum:
                self._curriculum(c)
            elif c.selected:
                self._selected(c)
            else:
                self._randomized(c)
        self.heightsamples = self.height_field_raw
        if self.type == "trimesh":
            self.vertices, self.triangles = convert_heightfield_to_trimesh(
                self.height_field_raw, cfg.horizontal_scale, cfg.vertical_scale, cfg.slope_treshold)

    @staticmethod
    def _dims(c):
        c.proportions = [float(np.sum(c.terrain_proportions[:i + 1])) for i in range(len(c.terrain_proportions))]
        c.num_sub_terrains = c.num_rows * c.num_cols
        c.env_origins = np.zeros((c.num_rows, c.num_cols, 3))
        c.width_per_env_pixels = int(c.terrain_length / c.horizontal_scale)
        c.length_per_env_pixels = int(c.terrain_width / c.horizontal_scale)
        c.border = int(c.border_size / c.horizontal_scale)
        c.tot_cols = int(c.num_cols * c.width_per_env_pixels) + 2 * c.border
        c.tot_rows = int(c.num_rows * c.length_per_env_pixels) + 2 * c.border

    def _layout(self):
        c, e = self.cfg, self.eval_cfg
        self._dims(c)
        c.row_indices, c.col_indices = np.arange(c.tot_rows), np.arange(c.tot_cols)
        c.x_offset = c.rows_offset = 0
        if e is None:
            return c.row_indices, c.col_indices, [], []
        self._dims(e)  # the eval tiles sit below the train tiles (rows offset)
        e.row_indices = np.arange(c.tot_rows, c.tot_rows + e.tot_rows)
        e.col_indices = np.arange(e.tot_cols)
        e.x_offset, e.rows_offset = c.tot_rows, c.num_rows
        return c.row_indices, c.col_indices, e.row_indices, e.col_indices

    def _randomized(self, c):
        for k in range(c.num_sub_terrains):
            i, j = np.unravel_index(k, (c.num_rows, c.num_cols))
            choice = np.random.uniform(0, 1)
            difficulty = np.random.choice([0.5, 0.75, 0.9])
            self._place(c, self._make(c, choice, difficulty, c.proportions), i, j)

    def _curriculum(self, c):
        for j in range(c.num_cols):
            for i in range(c.num_rows):
                difficulty = i / c.num_rows * c.difficulty_scale
                choice = j / c.num_cols + 0.001
                self._place(c, self._make(c, choice, difficulty, c.proportions), i, j)

    def _selected(self, c):
        kwargs = dict(c.terrain_kwargs)
        kind = kwargs.pop("type")
        fn = globals()[kind.split(".")[-1]]
        for k in range(c.num_sub_terrains):
            i, j = np.unravel_index(k, (c.num_rows, c.num_cols))
            t = SubTerrain("terrain", width=c.width_per_env_pixels, length=c.width_per_env_pixels,
                           vertical_scale=c.vertical_scale, horizontal_scale=c.horizontal_scale)
            fn(t, **kwargs.get("terrain_kwargs", {}))
            self._place(c, t, i, j)

    def _make(self, c, choice, difficulty, p):
        """terrain.py:113-163: the tile type by ``choice`` against the cumulative proportions."""
        t = SubTerrain("terrain", width=c.width_per_env_pixels, length=c.width_per_env_pixels,
                       vertical_scale=c.vertical_scale, horizontal_scale=c.horizontal_scale)
        slope = difficulty * 0.4
        step_height = 0.05 + 0.18 * difficulty
        obstacle_height = 0.05 + difficulty * (c.max_platform_height - 0.05)
        stone_size = 1.5 * (1.05 - difficulty)
        stone_distance = 0.05 if difficulty == 0 else 0.1
        bound = lambda k: p[k] if k < len(p) else float("inf")
        if choice < bound(0):
            pyramid_sloped_terrain(t, slope=-slope if choice < bound(0) / 2 else slope, platform_size=3.0)
        elif choice < bound(1):
            pyramid_sloped_terrain(t, slope=slope, platform_size=3.0)
            random_uniform_terrain(t, min_height=-0.05, max_height=0.05, step=self.cfg.terrain_smoothness,
                                   downsampled_scale=0.2)
        elif choice < bound(3):
            pyramid_stairs_terrain(t, step_width=0.31, step_height=-step_height if choice < bound(2) else step_height,
                                   platform_size=3.0)
        elif choice < bound(4):
            discrete_obstacles_terrain(t, obstacle_height, 1.0, 2.0, 20, platform_size=3.0)
        elif choice < bound(5):
            stepping_stones_terrain(t, stone_size=stone_size, stone_distance=stone_distance, max_height=0.0,
                                    platform_size=4.0)
        elif choice < bound(7):
            pass  # types 6 and 7: flat
        elif choice < bound(8):
            random_uniform_terrain(t, min_height=-c.terrain_noise_magnitude, max_height=c.terrain_noise_magnitude,
                                   step=0.005, downsampled_scale=0.2)
        elif choice < bound(9):
            random_uniform_terrain(t, min_height=-0.05, max_height=0.05, step=self.cfg.terrain_smoothness,
                                   downsampled_scale=0.2)
            t.height_field_raw[0:t.length // 2, :] = 0
        return t

    def _place(self, c, t, i, j):
        """terrain.py:165-184: copy the tile into the map, the tile's env origin = its centre at the height
        of the tile's highest point."""
        r0 = c.border + i * c.length_per_env_pixels + c.x_offset
        r1 = c.border + (i + 1) * c.length_per_env_pixels + c.x_offset
        c0 = c.border + j * c.width_per_env_pixels
        c1 = c.border + (j + 1) * c.width_per_env_pixels
        self.height_field_raw[r0:r1, c0:c1] = t.height_field_raw
        ox = (i + 0.5) * c.terrain_length + c.x_offset * t.horizontal_scale
        oy = (j + 0.5) * c.terrain_width
        oz = np.max(self.height_field_raw[r0:r1, c0:c1]) * t.vertical_scale
        c.env_origins[i, j] = [ox, oy, oz]

    def heights_m(self):
        """The device ground: float32 metres, [tot_rows, tot_cols]."""
        return (self.height_field_raw.astype(np.float32) * np.float32(self.cfg.vertical_scale)).astype(np.float32)
