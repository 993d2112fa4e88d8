"""Local-filesystem stand-in for ``ml_logger`` (the un-vendored experiment logger the reference imports:
scripts/train.py:11,38, scripts/play.py:18,74,93, mini_gym_learn/ppo/__init__.py:7,93-265).

``from ml_logger import logger`` gives the module-level :class:`ML_Logger` with the calls the reference makes —
``configure``, ``prefix``, ``utcnow``, ``log_text``, ``log_params``, ``start`` / ``since`` / ``split`` / ``every``,
``Prefix`` / ``Sync``, ``store_metrics`` / ``log_metrics_summary``, ``save_pkl`` / ``load_pkl``, ``torch_save`` /
``load_torch`` / ``duplicate`` / ``upload_file``, ``save_video``, ``glob`` and ``job_running`` — writing under a local
run directory instead of an instrument server.  Until ``configure`` names a directory nothing is written (metrics are
kept in memory), which is how the tests and ``bench.py`` run the Runner.
"""
import datetime
import glob as _glob
import os
import pickle
import shutil
import textwrap
import time
from collections import defaultdict
from collections.abc import Mapping
from contextlib import contextmanager

import numpy as np

__all__ = ["ML_Logger", "logger"]


def _plain(v, depth=0):
    """Parameters as plain data: class attributes (params_proto-style configs) become dicts, callables / dunders drop."""
    if isinstance(v, (bool, int, float, str, type(None))):
        return v
    if isinstance(v, (list, tuple)):
        return type(v)(_plain(x, depth + 1) for x in v)
    if isinstance(v, Mapping):
        return {str(k): _plain(x, depth + 1) for k, x in v.items()
                if not str(k).startswith("__") and (not callable(x) or isinstance(x, type))}
    if (isinstance(v, type) or (hasattr(v, "__dict__") and not callable(v))) and depth < 8:  # config classes / nodes
        return {k: _plain(x, depth + 1) for k, x in vars(v).items()
                if not k.startswith("__") and (not callable(x) or isinstance(x, type))}
    if hasattr(v, "tolist"):
        return v.tolist()
    return repr(v)


class ML_Logger:
    def __init__(self):
        self.prefix = None      # run path (relative to root when root is given), as ml_logger's logger.prefix
        self.root = None
        self.metrics = defaultdict(list)
        self.summaries = []
        self._metrics_prefix = ""
        self._timers = {}
        self._every = defaultdict(int)

    # ---- run directory ----
    @property
    def run_dir(self):
        if not self.prefix:
            return None
        return os.path.join(str(self.root), str(self.prefix)) if self.root else str(self.prefix)

    def configure(self, prefix=None, root=None, **_):
        self.prefix = str(prefix) if prefix is not None else None
        self.root = str(root) if root is not None else None
        if self.run_dir:
            os.makedirs(self.run_dir, exist_ok=True)
        return self

    def _path(self, path):
        d = self.run_dir
        if d is None:
            return None
        full = os.path.join(d, path)
        os.makedirs(os.path.dirname(full) or d, exist_ok=True)
        return full

    @staticmethod
    def utcnow(fmt="%Y-%m-%d/%H-%M-%S.%f"):
        return datetime.datetime.now(datetime.timezone.utc).strftime(fmt)

    def glob(self, pattern, wd=None):
        d = self.run_dir if wd is None else wd
        if d is None:
            return []
        return sorted(os.path.relpath(p, d) for p in _glob.glob(os.path.join(d, pattern)))

    def job_running(self, *_, **__):
        return None

    # ---- text / parameters / pickles ----
    def log_text(self, text, filename="text.log", dedent=False, overwrite=False):
        p = self._path(filename)
        if p is None:
            return
        if dedent:
            text = textwrap.dedent(text)
        with open(p, "w" if overwrite else "a") as f:
            f.write(text)

    def log_params(self, path="parameters.pkl", **kwargs):
        self.save_pkl({k: _plain(v) for k, v in kwargs.items()}, path=path, append=True)

    def save_pkl(self, data, path=None, append=False):
        p = self._path(path or "data.pkl")
        if p is None:
            return
        with open(p, "ab" if append else "wb") as f:
            pickle.dump(data, f)

    def load_pkl(self, path):
        """Every object ``save_pkl`` wrote to ``path`` (appended records in order), as ml_logger returns them."""
        p = self._path(path)
        out = []
        if p is None or not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            while True:
                try:
                    out.append(pickle.load(f))  # (a file this logger wrote)
                except EOFError:
                    break
        return out

    # ---- torch files ----
    def torch_save(self, obj, path):
        p = self._path(path)
        if p is None:
            return
        import torch
        torch.save(obj, p)

    save_torch = torch_save

    def load_torch(self, path, map_location=None):
        import torch
        return torch.load(self._path(path), map_location=map_location, weights_only=True)

    def duplicate(self, src, dst):
        s, d = self._path(src), self._path(dst)
        if s is not None and os.path.exists(s):
            shutil.copyfile(s, d)

    def upload_file(self, file_path, target_path="files/", once=False):
        d = self._path(os.path.join(target_path, os.path.basename(file_path)))
        if d is not None and os.path.abspath(d) != os.path.abspath(file_path):
            shutil.copyfile(file_path, d)

    def save_video(self, frames, key, fps=None, **_):
        """No video encoder in this image: the frames are kept as an ``.npz`` (frames [T, H, W, C], fps) next to
        where the reference's mp4 would go."""
        p = self._path(os.path.splitext(key)[0] + ".npz")
        if p is not None and len(frames):
            np.savez_compressed(p, frames=np.stack([np.asarray(f) for f in frames]), fps=np.float64(fps or 0.0))

    # ---- timers ----
    def start(self, *keys):
        t = time.time()
        for k in keys or ("default",):
            self._timers[k] = t
        return t

    def since(self, key="default"):
        t0 = self._timers.setdefault(key, time.time())
        return time.time() - t0

    def split(self, key="default"):
        t = time.time()
        t0 = self._timers.get(key, t)
        self._timers[key] = t
        return t - t0

    def every(self, n=1, key="default", start_on=0):
        """True on calls start_on, start_on + n, ... of ``key`` (counted from 1, as ml_logger counts)."""
        self._every[key] += 1
        c = self._every[key]
        return n > 0 and c >= start_on and (c - start_on) % n == 0

    # ---- metrics ----
    @contextmanager
    def Prefix(self, *praefixa, metrics=None):
        old = self._metrics_prefix
        if metrics is not None:
            self._metrics_prefix = os.path.join(old, metrics) if old else metrics
        try:
            yield self
        finally:
            self._metrics_prefix = old

    @contextmanager
    def Sync(self, *_, **__):
        yield self

    def store_metrics(self, metrics=None, **kwargs):
        kv = dict(metrics or {}, **kwargs)
        for k, v in kv.items():
            key = f"{self._metrics_prefix}/{k}" if self._metrics_prefix else k
            # (device scalars are kept as they are and converted when summarised: no host sync per store)
            self.metrics[key].append(v)

    def log_metrics_summary(self, key_values=None, default_stats="mean", **_):
        """``{key}/{stat}`` over everything stored since the last summary, plus ``key_values``; device scalars (the
        Runner stores its losses and episode means without a host sync) are reduced on their device and fetched in one
        copy, not one sync per stored value."""
        s, dev_keys, dev_stats = {}, [], []
        for k, vs in self.metrics.items():
            if not vs:
                continue
            tens = [v for v in vs if hasattr(v, "detach")]
            if tens and len(tens) == len(vs):
                import torch
                t = torch.stack([v.detach().reshape(()).to(torch.float64) for v in tens])
                dev_keys.append(k)
                dev_stats.append(getattr(torch, default_stats)(t))
            else:
                arr = np.array([float(v) for v in vs], dtype=np.float64)
                s[f"{k}/{default_stats}"] = float(getattr(np, default_stats)(arr))
        if dev_stats:
            import torch
            by_dev = {}
            for k, v in zip(dev_keys, dev_stats):
                by_dev.setdefault(v.device, []).append((k, v))
            for items in by_dev.values():
                vals = torch.stack([v for _, v in items]).tolist()  # (one device -> host copy per device)
                for (k, _), x in zip(items, vals):
                    s[f"{k}/{default_stats}"] = float(x)
        s.update(key_values or {})
        self.summaries.append(s)
        self.metrics.clear()
        self.save_pkl(s, path="metrics.pkl", append=True)
        return s

    def log_metrics(self, metrics=None, **kwargs):
        s = dict(metrics or {}, **kwargs)
        self.summaries.append(s)
        self.save_pkl(s, path="metrics.pkl", append=True)


logger = ML_Logger()
