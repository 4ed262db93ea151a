"""Drop-in model classes for the GCN hot path, with the reference's API and ``state_dict`` keys.

Mirrors ``dgl/model/models.py``:

* :class:`edge_encoder`  — ``models.py:142-155``: ``Linear(9,C) -> ReLU -> Linear(C,2C) -> Sigmoid``;
  keys ``layers.0.weight``, ``layers.0.bias``, ``layers.2.weight``, ``layers.2.bias``.
* :class:`GCN`           — ``models.py:213-226``: ``forward(g)`` (the reference call, ``models.py:181``)
  and ``forward(g, feats)`` (the north-star signature).  Aggregation runs in the HIP kernel.
* :class:`GCNBlock`      — the GCN stacking of ``multi_view_dgl_model.forward`` (``models.py:180-189``):
  ``gcn1 -> cat -> [conv1] -> [gcn2 -> cat -> conv2]``, keys ``gcn1.*``, ``conv1.*``, ``gcn2.*``, ``conv2.*``;
  the 1x1 convs run on the matrix-core compress kernels without the concatenation (``compress.py``).
* :class:`GCNStack`      — the same for k layers (``opt.gcn_layers``; BASELINE configs[4] runs 3) and
  the residual (``dgl_models.py:36-37``) / initial-feature-mix combinations, each fused into the
  aggregation kernel's epilogue.
* :class:`multi_view_dgl_model` — ``models.py:157-205`` with the CNN encoder/decoder supplied by the
  caller (they are torchvision/dense-conv code outside the hot path), so a reference
  ``encoder``/``decoder`` instance can be plugged in unchanged.

Semantics switch ``opt.gcn_return``:

* ``'aggregate'`` (default): return the FiLM-mean aggregate — what ``update_all`` computes and
  what the scratch variants return (``dgl/model/dgl_models.py:61,127,189``).
* ``'input'``: bit-faithful to ``models.py:226``, which returns ``g.ndata['image']`` (the input)
  because ``node_udf`` writes ``'images'``; the aggregate is then dead work and is skipped.

``opt.gcn_mode``: ``'film_mean'`` (default, ``models.py:223``), ``'copy_mean'`` (the commented-out
``fn.copy_u`` variant, ``models.py:225``), ``'film_sum'``.
"""
from __future__ import annotations

import warnings

import torch
import torch.nn as nn

from .aggregate import film_mean, film_mean_cat, film_mean_mix, film_mean_residual
from .compress import compress_1x1, compress_path, film_compress, film_compress_supported
from .encoder import edge_logits


def clear_packed_weights() -> None:
    """Drop every cached split-bf16 weight image (edge encoder and 1x1 compress).  The images are
    keyed by a weight's data pointer and autograd version, which in-place optimizer steps bump;
    writes that bypass the version counter (``param.data = t``, ``.data`` copies, collectives
    writing into parameters) need this call.  The modules below call it themselves when they are
    moved or cast (``.to()``, ``.cuda()``, ``.float()``: ``nn.Module._apply``) and after
    ``load_state_dict``."""
    from . import compress, encoder
    compress.clear_packed_weights()
    encoder.clear_packed_weights()


class _PackedImages:
    """Mixin: invalidate the packed weight images when parameters are replaced wholesale."""

    def _apply(self, fn, *args, **kwargs):
        clear_packed_weights()
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        out = super().load_state_dict(*args, **kwargs)
        clear_packed_weights()
        return out


class edge_encoder(_PackedImages, nn.Module):  # noqa: N801  (reference class name)
    """FiLM parameter generator, ``dgl/model/models.py:142-155``."""

    def __init__(self, layers_dim):
        super().__init__()
        self.layers_dim = layers_dim
        self.layers = nn.Sequential(
            nn.Linear(9, layers_dim[0]),
            nn.ReLU(),
            nn.Linear(layers_dim[0], layers_dim[1] * 2),
            nn.Sigmoid(),
        )

    def logits(self, edge: torch.Tensor) -> torch.Tensor:
        """Pre-sigmoid FiLM parameters z, (E, C, 2) interleaved.  On the GPU (``encoder.edge_logits``):
        one split-bf16 matrix-core kernel for both Linears (``mrp_edge_encoder_fwd_split``); with a
        gradient wanted the same kernel also keeps h^T for a backward on the split-bf16 GEMM kernels.
        The sigmoid is left to the aggregation kernel (``MRP_AGG_GB_LOGITS``)."""
        if edge.is_cuda:
            z = edge_logits(self.layers, edge)
        else:
            z = self.layers[2](self.layers[1](self.layers[0](edge.float())))
        return z.view(-1, self.layers_dim[1], 2)

    def film_params(self, edge: torch.Tensor) -> torch.Tensor:
        """Interleaved gamma/beta = sigmoid(z), (E, C, 2) (``models.py:153-154``)."""
        return torch.sigmoid(self.logits(edge))

    def forward(self, edge: torch.Tensor):
        """Reference return value: gamma, beta as (E, C, 1, 1) views (``models.py:152-155``)."""
        gb = self.film_params(edge)
        return gb[:, :, 0].unsqueeze(-1).unsqueeze(-1), gb[:, :, 1].unsqueeze(-1).unsqueeze(-1)


def _opt(opt, name, default):
    return getattr(opt, name, default) if opt is not None else default


#: ``gcn_return`` given to a GCN unpickled from a reference checkpoint whose ``opt`` has none (see
#: :meth:`GCN.__setstate__`); ``compat.reference_class_path(gcn_return=...)`` sets it.
UNPICKLED_GCN_RETURN = "input"


class GCN(_PackedImages, nn.Module):
    """FiLM-mean graph convolution over per-frame robot graphs, ``dgl/model/models.py:213-226``."""

    def __init__(self, opt):
        super().__init__()
        self.opt = opt
        self.edge_encoder = edge_encoder(layers_dim=[opt.feature_dim, opt.feature_dim])
        # marks a GCN this framework built: its pickles (deepcopy, torch.save of the whole model as the
        # reference's training.py:345-355 does) keep computing the aggregate
        self.gcn_return_default = "aggregate"

    def __setstate__(self, state):
        """Unpickling a checkpoint the reference wrote (``torch.save({'model': model})``,
        ``dgl/training.py:345-355``): its ``opt`` has no ``gcn_return``, and the reference forward
        it was trained and evaluated with returns its input (``models.py:226``).  Keep that
        behaviour so ``eval.py`` reproduces the reference's outputs, and say so once.  A GCN built
        here carries ``gcn_return_default`` in its state and keeps it."""
        super().__setstate__(state)
        if self.__dict__.get("opt") is not None and not hasattr(self.opt, "gcn_return") \
                and "gcn_return_default" not in self.__dict__:
            self.gcn_return_default = UNPICKLED_GCN_RETURN
            if UNPICKLED_GCN_RETURN == "input":
                warnings.warn("mrp_gnn: GCN unpickled from a checkpoint without opt.gcn_return: returning the "
                              "input as the reference's GCN.forward does (models.py:226); set "
                              "opt.gcn_return='aggregate' for the message-passing result", stacklevel=2)

    def _return_mode(self) -> str:
        return _opt(self.opt, "gcn_return", self.__dict__.get("gcn_return_default", "aggregate"))

    def forward(self, g, feats: torch.Tensor = None) -> torch.Tensor:
        x = g.ndata["image"] if feats is None else feats
        if self._return_mode() == "input":
            return x  # models.py:226 returns the input; update_all's result is never read
        mode = _opt(self.opt, "gcn_mode", "film_mean")
        if mode == "copy_mean":
            return film_mean(x, None, g.csr(x.device), mode)
        # logits in, sigmoid applied inside the aggregation kernel
        z = self.edge_encoder.logits(g.edata["pose"])
        return film_mean(x, z, g.csr(x.device), mode, logits=True)

    def forward_cat(self, g, feats: torch.Tensor = None) -> torch.Tensor:
        """``torch.cat((feats, self(g, feats)), 1)`` (``models.py:181-182``) with the aggregate written
        straight into the concatenation buffer (and the backward fused likewise)."""
        x = g.ndata["image"] if feats is None else feats
        if self._return_mode() == "input" or not x.is_cuda:
            return torch.cat((x, self(g, x)), dim=1)
        mode = _opt(self.opt, "gcn_mode", "film_mean")
        if mode == "copy_mean":
            return film_mean_cat(x, None, g.csr(x.device), mode)
        z = self.edge_encoder.logits(g.edata["pose"])
        return film_mean_cat(x, z, g.csr(x.device), mode, logits=True)


    def forward_cat_compress(self, g, feats: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
        """``conv(torch.cat((feats, self(g, feats)), 1))`` (``models.py:181-184``) without the
        concatenation: the aggregation kernel into its own buffer, then the matrix-core compress
        reading x and the aggregate in place, and in backward the data-gradient kernel writing x's
        gradient half and the aggregate's gradient straight into the aggregation backward, plus the
        split-K weight-gradient kernel (``compress.FilmCompressFunction``).  With
        ``compress.set_compress_path('library')``: the cat kernel + torch's library GEMMs."""
        x = feats
        if (x.is_cuda and self._return_mode() != "input" and compress_path() != "library"
                and film_compress_supported(conv, x)):
            mode = _opt(self.opt, "gcn_mode", "film_mean")
            if mode == "copy_mean":
                return film_compress(conv, x, None, g.csr(x.device), _lib_modes()[mode])
            z = self.edge_encoder.logits(g.edata["pose"])
            return film_compress(conv, x, z, g.csr(x.device), _lib_modes()[mode] | _lib_logits())
        return compress_1x1(conv, self.forward_cat(g, x))

    def forward_residual(self, g, feats: torch.Tensor = None) -> torch.Tensor:
        """``feats + self(g, feats)`` in one kernel pass: the residual combination ``h = g_h + h``
        of ``dgl/model/dgl_models.py:36-37`` (the FiLM-mean 'add' variant)."""
        x = g.ndata["image"] if feats is None else feats
        if self._return_mode() == "input" or not x.is_cuda:
            return x + self(g, x)
        mode = _opt(self.opt, "gcn_mode", "film_mean")
        if mode == "copy_mean":
            return film_mean_residual(x, None, g.csr(x.device), mode)
        z = self.edge_encoder.logits(g.edata["pose"])
        return film_mean_residual(x, z, g.csr(x.device), mode, logits=True)

    def forward_mix(self, g, feats: torch.Tensor, x0: torch.Tensor, alpha: float) -> torch.Tensor:
        """``(1 - alpha) * self(g, feats) + alpha * x0`` in one kernel pass: a GCN2-style
        initial-feature mix (BASELINE configs[3]'s "GCN2Conv"; not in the reference)."""
        x = feats
        if self._return_mode() == "input" or not x.is_cuda:
            return (1.0 - alpha) * self(g, x) + alpha * x0
        mode = _opt(self.opt, "gcn_mode", "film_mean")
        if mode == "copy_mean":
            return film_mean_mix(x, None, g.csr(x.device), x0, alpha, mode)
        z = self.edge_encoder.logits(g.edata["pose"])
        return film_mean_mix(x, z, g.csr(x.device), x0, alpha, mode, logits=True)


def _lib_modes():
    from . import _lib
    return _lib.MODES


def _lib_logits():
    from . import _lib
    return _lib.GB_LOGITS


#: layer compositions of a GCN stack (``GCNStack``, ``multi_view_dgl_model``)
COMBINES = ("cat_compress", "cat", "residual", "initial_mix")


def stack_layout(opt):
    """(number of GCN layers, combine, 1x1 compress convs?) from the reference flags
    (``compress_gcn``, ``multi_gcn``, ``models.py:162-171``) or their generalisation
    ``opt.gcn_layers`` / ``opt.gcn_combine``:

    * ``'cat_compress'`` — ``h = conv_i(cat(h, gcn_i(h)))`` per layer (``models.py:180-189``;
      ``multi_gcn`` is two such layers; k layers extend the ``gcn<i>``/``conv<i>`` naming);
    * ``'cat'`` — one layer, ``h = cat(h, gcn1(h))`` (2C channels; ``compress_gcn`` off);
    * ``'residual'`` — ``h = h + gcn_i(h)`` (``dgl_models.py:36-37``), no convs;
    * ``'initial_mix'`` — ``h = (1 - alpha) gcn_i(h) + alpha h0`` (``opt.gcn2_alpha``, default 0.1;
      GCN2-style extension, not in the reference), no convs."""
    layers = int(_opt(opt, "gcn_layers", 0) or (2 if _opt(opt, "multi_gcn", False) else 1))
    combine = _opt(opt, "gcn_combine", None)
    if combine is None:
        combine = "cat_compress" if _opt(opt, "compress_gcn", False) else "cat"
    if combine not in COMBINES:
        raise ValueError(f"gcn_combine must be one of {COMBINES}, got {combine!r}")
    if layers < 1:
        raise ValueError("gcn_layers must be >= 1")
    if combine == "cat" and layers > 1:
        raise AssertionError("stacked GCN layers need compress_gcn (models.py:169)")
    return layers, combine, combine == "cat_compress"


def _build_stack(module: nn.Module, opt) -> None:
    layers, combine, convs = stack_layout(opt)
    module.gcn_layers, module.gcn_combine = layers, combine
    for i in range(1, layers + 1):
        setattr(module, f"gcn{i}", GCN(opt))
        if convs:
            setattr(module, f"conv{i}", nn.Conv2d(opt.feature_dim * 2, opt.feature_dim, kernel_size=1))


def _run_stack(module: nn.Module, g, h: torch.Tensor) -> torch.Tensor:
    """The layer loop of ``multi_view_dgl_model.forward`` (``models.py:180-189``), k layers."""
    h0 = h
    alpha = float(_opt(module.opt, "gcn2_alpha", 0.1))
    for i in range(1, module.gcn_layers + 1):
        gcn = getattr(module, f"gcn{i}")
        if module.gcn_combine == "cat_compress":
            h = gcn.forward_cat_compress(g, h, getattr(module, f"conv{i}"))  # conv_i(cat((h, gcn_i(h)), 1))
        elif module.gcn_combine == "cat":
            h = gcn.forward_cat(g, h)  # cat((h, gcn_i(h)), 1), one kernel pass
        elif module.gcn_combine == "residual":
            h = gcn.forward_residual(g, h)
        else:
            h = gcn.forward_mix(g, h, h0, alpha)
    return h


class GCNStack(_PackedImages, nn.Module):
    """k stacked GCN layers (``dgl/model/models.py:162-171,180-189`` generalised; see
    :func:`stack_layout`).  ``state_dict`` keys ``gcn1.*``, ``conv1.*``, ..., ``gcn<k>.*``,
    ``conv<k>.*`` — the reference's naming for k = 1, 2."""

    def __init__(self, opt):
        super().__init__()
        self.opt = opt
        _build_stack(self, opt)

    def forward(self, g, h: torch.Tensor) -> torch.Tensor:
        return _run_stack(self, g, h)


class GCNBlock(GCNStack):
    """GCN stacking of ``multi_view_dgl_model`` (``dgl/model/models.py:162-171,180-189``): gcn1 ->
    cat -> [conv1] -> [gcn2 -> cat -> conv2] from the reference's ``compress_gcn``/``multi_gcn``
    flags (a :class:`GCNStack` of one or two layers)."""

    def __init__(self, opt):
        if opt.multi_gcn:
            assert opt.compress_gcn  # models.py:169
        super().__init__(opt)


class multi_view_dgl_model(_PackedImages, nn.Module):  # noqa: N801  (reference class name)
    """``dgl/model/models.py:157-205`` with caller-supplied CNN ``encoder``/``decoder``.

    ``encoder(images (B, N, 3, S, S)) -> list of feature maps`` (last one used) and
    ``decoder(h) -> prediction`` follow the reference modules' call signatures; with
    ``encoder=None`` the node features in ``g.ndata['image']`` are taken to be feature maps
    already (the synthetic benchmark setting).
    """

    def __init__(self, opt, encoder: nn.Module = None, decoder: nn.Module = None):
        super().__init__()
        self.opt = opt
        if encoder is not None:
            self.encoder = encoder
        if _opt(opt, "multi_gcn", False):
            assert opt.compress_gcn  # models.py:169
        _build_stack(self, opt)  # gcn1 [conv1] [gcn2 conv2] ... (models.py:162-171)
        if decoder is not None:
            self.decoder = decoder

    def __setstate__(self, state):
        super().__setstate__(state)
        if "gcn_layers" not in self.__dict__:  # pickled by the reference: its flags give the layout
            self.gcn_layers, self.gcn_combine, _ = stack_layout(self.opt)

    def features(self, g):
        """Encoder output per node, (B*N, C, h, w), and the encoder's feature list
        (``models.py:175-179``)."""
        image = g.ndata["image"]
        if not hasattr(self, "encoder"):
            return image, [image]
        image = image.view(-1, self.opt.camera_num, 3, self.opt.image_size, self.opt.image_size)
        h_list = self.encoder(image)
        h = h_list[-1]
        return h.view(-1, h.size()[-3], h.size()[-2], h.size()[-1]), h_list

    def decode(self, h, h_list):
        """The decoder heads of ``models.py:190-205``: ``skip_level`` also passes the encoder's
        feature list; ``task='depthseg'`` calls ``depth_decoder`` and ``seg_decoder``."""
        if _opt(self.opt, "task", "depth") == "depthseg" and hasattr(self, "depth_decoder"):
            heads = (self.depth_decoder, self.seg_decoder)
        elif hasattr(self, "decoder"):
            heads = (self.decoder,)
        else:
            return h  # no decoder supplied: the GCN block's output (the benchmark setting)
        args = (h, h_list) if _opt(self.opt, "skip_level", False) else (h,)
        outs = tuple(head(*args) for head in heads)
        return outs if len(outs) > 1 else outs[0]

    def forward(self, g):
        with g.local_scope():
            h, h_list = self.features(g)
            g.ndata["image"] = h
            h = _run_stack(self, g, h)  # gcn1 -> cat -> conv1 [-> gcn2 -> cat -> conv2], models.py:180-189
            return self.decode(h, h_list)
