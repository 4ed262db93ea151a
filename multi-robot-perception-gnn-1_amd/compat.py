"""Drop-in compatibility with the reference harness (``dgl/training.py``, ``dgl/eval.py``).

The reference harness touches this path through two imports and one file format:

* ``from model import models`` (``dgl/training.py:13``) and ``models.multi_view_dgl_model(opt)``
  (``:303-304``); checkpoints are whole pickled modules, ``torch.save({'model': model, ...})``
  (``dgl/training.py:339-355``), reloaded with ``checkpoint['model']`` (``dgl/training.py:289-291``,
  ``dgl/eval.py:251-252``).  Unpickling resolves classes by their path ``model.models.<name>``.
* ``from dgl import batch`` as the DataLoader collate (``dgl/training.py:15,57-58``,
  ``dgl/eval.py:12,55-56``) and ``data.to('cuda:0')`` on its result.

:func:`install` registers two import aliases so that both work on top of this package:

* ``model.models`` — ``GCN``, ``edge_encoder`` and ``multi_view_dgl_model`` resolve to the
  MI355X classes (identical attribute names and ``state_dict`` keys, so a reference checkpoint
  unpickles straight into them); every other name (the torchvision ``encoder``, ``decoder``,
  ``TransBlock``, the non-graph baselines — outside the hot path) is looked up in ``fallback``,
  the caller's own import of the reference ``models`` module, if one is given.
* ``dgl`` (only when the real DGL is not importable) — ``batch``, ``unbatch``, ``graph`` and
  ``DGLGraph`` backed by :class:`~graph.RobotGraph`; ``save_graphs``/``load_graphs`` for the dataset's
  graph cache (``dgl/dataloader.py:165-175``; this package's own ``.npz``-based format — DGL's
  binary format is not read, a DGL-written cache is rebuilt); ``dgl.data.DGLDataset``, the base
  class of the reference's ``MultiViewDGLDataset``.

With the aliases installed, the reference's own ``train_dgl``/``test_dgl`` loops run unchanged:
the collate yields a :class:`~graph.RobotGraph`, ``.to('cuda:0')`` moves its features, and the
model's GCN layers run the HIP kernels.  Loading pickles executes code from the file: only load
checkpoints you trust (``torch.load(..., weights_only=False)``); for untrusted files use
``state_dict`` loading — the keys are identical (``tests/test_compat.py``).
"""
from __future__ import annotations

import contextlib
import importlib.util
import os
import sys
import types
from typing import Optional

from . import graph as _graph
from . import models as _models

#: names the aliased ``model.models`` serves from this package
NATIVE_CLASSES = ("GCN", "edge_encoder", "multi_view_dgl_model")


def collate(graphs):
    """The harness's ``_collate_fn`` (``dgl/training.py:57-58``): ``dgl.batch`` of frame graphs."""
    return _graph.batch(graphs)


def models_module(fallback: Optional[types.ModuleType] = None) -> types.ModuleType:
    """A module object standing in for the reference's ``model.models``."""
    mod = types.ModuleType("model.models")
    mod.__doc__ = "mrp_gnn_amd alias of the reference's dgl/model/models.py (hot-path classes native)"
    for name in NATIVE_CLASSES:
        setattr(mod, name, getattr(_models, name))

    def __getattr__(name):  # PEP 562: reference-only classes come from the caller's fallback
        if fallback is not None and hasattr(fallback, name):
            return getattr(fallback, name)
        raise AttributeError(
            f"model.models.{name} is outside the MI355X hot path; pass the reference module as "
            f"install(fallback=...) to resolve it")

    mod.__getattr__ = __getattr__
    return mod


class DGLDataset:
    """The ``dgl.data.DGLDataset`` lifecycle the reference dataset subclasses
    (``dgl/dataloader.py:15-60,165-202``): the constructor records ``name``/``url``/``raw_dir``/
    ``save_dir``/``force_reload``/``verbose`` and then loads — ``load()`` if ``has_cache()`` (and not
    ``force_reload``), else ``download()``, ``process()``, ``save()``.  Restated from DGL's documented
    behaviour (DGL itself is absent)."""

    def __init__(self, name, url=None, raw_dir=None, save_dir=None, hash_key=(), force_reload=False,
                 verbose=False):
        self._name = name
        self._url = url
        self._raw_dir = raw_dir if raw_dir is not None else os.path.join(os.path.expanduser("~"), ".dgl")
        self._save_dir = save_dir if save_dir is not None else self._raw_dir
        self._hash_key = hash_key
        self._force_reload = force_reload
        self._verbose = verbose
        self._load()

    # the subclass API
    def download(self):
        pass

    def process(self):
        raise NotImplementedError

    def save(self):
        pass

    def load(self):
        pass

    def has_cache(self):
        return False

    def __getitem__(self, idx):
        raise NotImplementedError

    def __len__(self):
        raise NotImplementedError

    # DGL's properties
    @property
    def name(self):
        return self._name

    @property
    def url(self):
        return self._url

    @property
    def raw_dir(self):
        return self._raw_dir

    @property
    def save_dir(self):
        return self._save_dir

    @property
    def raw_path(self):
        return os.path.join(self._raw_dir, self._name)

    @property
    def save_path(self):
        return os.path.join(self._save_dir, self._name)

    @property
    def verbose(self):
        return self._verbose

    def _load(self):
        loaded = False
        if not self._force_reload and self.has_cache():
            try:
                self.load()
                loaded = True
            except (OSError, ValueError, KeyError) as e:  # stale / foreign cache: rebuild it
                if self._verbose:
                    print(f"[{self._name}] cache not loadable ({e}); processing again")
        if not loaded:
            os.makedirs(self._raw_dir, exist_ok=True)
            self.download()
            self.process()
            os.makedirs(self._save_dir, exist_ok=True)
            self.save()


def dgl_module() -> types.ModuleType:
    """The slice of the ``dgl`` namespace the reference touches on this path: ``batch`` (collate),
    ``graph``, ``save_graphs``/``load_graphs`` (dataset cache, this package's own format),
    ``unbatch``, ``DGLGraph`` and ``dgl.data.DGLDataset``."""
    mod = types.ModuleType("dgl")
    mod.__doc__ = "mrp_gnn_amd stand-in for dgl (batch / graph / DGLGraph on RobotGraph)"
    mod.__path__ = []
    mod.batch = _graph.batch
    mod.unbatch = _graph.unbatch
    mod.graph = _graph.graph
    mod.save_graphs = _graph.save_graphs
    mod.load_graphs = _graph.load_graphs
    mod.DGLGraph = _graph.RobotGraph
    mod.data = types.ModuleType("dgl.data")
    mod.data.DGLDataset = DGLDataset
    return mod


def _dgl_importable() -> bool:
    mod = sys.modules.get("dgl")
    if mod is not None:
        return not getattr(mod, "__doc__", "").startswith("mrp_gnn_amd")
    return importlib.util.find_spec("dgl") is not None


def install(fallback: Optional[types.ModuleType] = None, dgl: bool = True) -> dict:
    """Register the ``model.models`` (and, if DGL is absent, ``dgl``) aliases in ``sys.modules``.
    Returns the previous entries, for :func:`uninstall`."""
    saved = {k: sys.modules.get(k) for k in ("model", "model.models", "dgl", "dgl.data")}
    pkg = types.ModuleType("model")
    pkg.__path__ = []  # a package, so ``from model import models`` and pickle's import both work
    pkg.models = models_module(fallback)
    sys.modules["model"] = pkg
    sys.modules["model.models"] = pkg.models
    if dgl and not _dgl_importable():
        sys.modules["dgl"] = dgl_module()
        sys.modules["dgl.data"] = sys.modules["dgl"].data
    return saved


def uninstall(saved: dict) -> None:
    for k, v in saved.items():
        if v is None:
            sys.modules.pop(k, None)
        else:
            sys.modules[k] = v


@contextlib.contextmanager
def reference_class_path(fallback: Optional[types.ModuleType] = None, dgl: bool = True,
                         gcn_return: str = "input"):
    """``with reference_class_path(): ckpt = torch.load(path, weights_only=False)`` — unpickle a
    reference checkpoint into the MI355X classes.

    A reference ``opt`` carries no ``gcn_return``; GCN layers unpickled here without one return
    ``gcn_return`` — by default ``'input'``, what the reference's ``GCN.forward`` returns
    (``models.py:226``), so the checkpoint's eval outputs are reproduced.  Pass
    ``gcn_return='aggregate'`` for the message-passing result (what the scratch variants return)."""
    if gcn_return not in ("input", "aggregate"):
        raise ValueError(f"gcn_return must be 'input' or 'aggregate', got {gcn_return!r}")
    saved = install(fallback, dgl)
    prev = _models.UNPICKLED_GCN_RETURN
    _models.UNPICKLED_GCN_RETURN = gcn_return
    try:
        yield sys.modules["model.models"]
    finally:
        _models.UNPICKLED_GCN_RETURN = prev
        uninstall(saved)
