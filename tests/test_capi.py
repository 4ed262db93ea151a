"""CPU: the C-ABI library loads and exports every symbol include/*.h declares; argument
validation and no-op paths (no compute launch, so no GPU needed); the product has no CPU fallback."""
import ctypes
import glob
import os
import re
import subprocess

import pytest
import torch

import mrp_gnn_amd as m
from mrp_gnn_amd import _lib
from conftest import ROOT

HIP_INVALID_VALUE = 1


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        syms |= set(re.findall(r"^\s*(?:int|int64_t|const char\*|void)\s+(mrp_\w+)\s*\(", text, re.M))
    return syms


def test_header_declares_expected_symbols():
    assert declared_symbols() == set(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = m.load_library()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (mrp_\w+)$", out, re.M))
    assert declared_symbols() == exported  # exactly the header's entry points: no lab hooks


def test_library_targets_gfx950_only():
    data = open(_lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-+(gfx\w+)", data))
    assert targets == {b"gfx950"}


def test_abi_version_and_errors():
    lib = m.load_library()
    assert lib.mrp_abi_version() == _lib.ABI_VERSION
    assert b"invalid" in lib.mrp_error_string(HIP_INVALID_VALUE).lower()


def _fwd(lib, **kw):
    a = dict(x=None, xs=0, gb=None, indptr=None, src=None, eid=None, goff=None, B=0, maxn=0, kind=0, Nt=0, E=0,
             C=0, P=0, mode=0, out=None, os=0, stream=None)
    a.update(kw)
    return lib.mrp_film_mean_fwd(a["x"], a["xs"], a["gb"], a["indptr"], a["src"], a["eid"], a["goff"], a["B"],
                                 a["maxn"], a["kind"], a["Nt"], a["E"], a["C"], a["P"], a["mode"], a["out"], a["os"],
                                 a["stream"])


def test_argument_validation_without_launch():
    lib = m.load_library()
    dummy = ctypes.c_void_p(16)
    assert _fwd(lib) == 0  # empty batch: no-op
    assert _fwd(lib, maxn=17, B=1, Nt=1, goff=dummy, indptr=dummy) == HIP_INVALID_VALUE  # > MRP_MAX_NODES
    assert _fwd(lib, mode=3) == HIP_INVALID_VALUE
    assert _fwd(lib, C=-1) == HIP_INVALID_VALUE
    # more nodes than num_graphs * max_nodes can hold
    assert _fwd(lib, B=1, maxn=2, Nt=3, goff=dummy, indptr=dummy) == HIP_INVALID_VALUE
    # stride smaller than a node's C*P block
    assert _fwd(lib, B=1, maxn=2, Nt=2, goff=dummy, indptr=dummy, C=2, P=4, x=dummy, out=dummy, xs=7, os=8,
                mode=2) == HIP_INVALID_VALUE
    # unknown graph kind; COMPLETE with inconsistent node / edge counts
    assert _fwd(lib, kind=2) == HIP_INVALID_VALUE
    assert _fwd(lib, kind=1, B=2, maxn=4, Nt=8, E=23) == HIP_INVALID_VALUE
    assert _fwd(lib, kind=1, B=2, maxn=4, Nt=7, E=24) == HIP_INVALID_VALUE
    assert _fwd(lib, kind=1, B=2, maxn=4, Nt=8, E=24, C=0, P=16) == 0  # consistent, empty features: no-op
    # bwd: nothing requested -> no-op
    assert lib.mrp_film_mean_bwd(None, 0, None, 0, None, None, None, None, None, 0, 0, 0, 0, 0, 0, 0, 0, None, 0,
                                 None, 0, None, None) == 0


def test_no_cpu_fallback():
    g = m.complete_graph(3)
    x = torch.randn(3, 2, 4, 4)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m.film_mean(x, torch.rand(6, 2, 2), g.csr("cpu"))


def test_frame_graph_build_validation_without_launch():
    lib = m.load_library()
    dummy = ctypes.c_void_p(16)
    # more robots per frame than MRP_MAX_NODES, k >= n, negative sizes: rejected before any launch
    assert lib.mrp_frame_graph_build(dummy, 1, 17, 0, dummy, dummy, dummy, dummy, dummy, None) == HIP_INVALID_VALUE
    assert lib.mrp_frame_graph_build(dummy, 1, 4, 4, dummy, dummy, dummy, dummy, dummy, None) == HIP_INVALID_VALUE
    assert lib.mrp_frame_graph_build(dummy, -1, 4, 0, dummy, dummy, dummy, dummy, dummy, None) == HIP_INVALID_VALUE
    assert lib.mrp_frame_graph_build(None, 2, 4, 0, None, None, None, None, None, None) == HIP_INVALID_VALUE


def test_frame_batch_needs_the_gpu():
    with pytest.raises(RuntimeError, match="GPU"):
        m.frame_batch(torch.zeros(2, 4, 7))


def test_edge_encoder_bwd_validation_without_launch():
    lib = m.load_library()
    assert lib.mrp_edge_encoder_bwd_workspace(1792, 512) == 112 * 12 * 512 * 4  # 16-edge chunks x 12C floats
    assert lib.mrp_film_mean_bwd_workspace(8, 16, m.graph_regular(4), 1024, 256) == 0  # reserved since ABI 12
    assert lib.mrp_edge_encoder_bwd_workspace(0, 512) == 0
    assert lib.mrp_edge_encoder_bwd(None, None, None, None, -1, 4, None, None, None, None, None) == HIP_INVALID_VALUE
    # work to do but a missing input or workspace
    assert lib.mrp_edge_encoder_bwd(None, None, None, None, 8, 4, None, None, None, None, None) == HIP_INVALID_VALUE
    assert lib.mrp_edge_encoder_bwd(None, None, None, None, 8, 0, None, None, None, None, None) == 0  # C = 0: no-op


def test_split_encoder_validation_without_launch():
    lib = m.load_library()
    # packed image: W1/b1 parts (C/32 x 3 x 64 lanes x 16 B) + W2 parts (2C/32 x C/32 x 2 x 3 x 64 x 16 B)
    assert lib.mrp_edge_encoder_pack_bytes(512) == 512 * 96 + 2 * 512 * 512 * 6
    assert lib.mrp_edge_encoder_pack_bytes(48) == 0 and lib.mrp_edge_encoder_pack_bytes(0) == 0
    assert lib.mrp_edge_encoder_pack(None, None, None, 48, None, None) == m._lib.HIP_ERROR_NOT_SUPPORTED
    assert lib.mrp_edge_encoder_pack(None, None, None, 64, None, None) == HIP_INVALID_VALUE
    assert lib.mrp_edge_encoder_fwd_split(None, None, None, 0, 64, None, None) == 0  # no edges: no-op
    assert lib.mrp_edge_encoder_fwd_split(None, None, None, 10, 48, None, None) == m._lib.HIP_ERROR_NOT_SUPPORTED
    assert lib.mrp_edge_encoder_fwd_split(None, None, None, 10, 64, None, None) == HIP_INVALID_VALUE
    assert lib.mrp_edge_encoder_fwd_split(None, None, None, -1, 64, None, None) == HIP_INVALID_VALUE
    # the image is addressed with 32-bit offsets: 96 C + 12 C^2 bytes must stay below 2^31 (C <= 13344)
    assert 96 * 13344 + 12 * 13344 ** 2 < 2 ** 31 <= 96 * 13376 + 12 * 13376 ** 2
    assert lib.mrp_edge_encoder_pack(None, None, None, 13376, None, None) == m._lib.HIP_ERROR_NOT_SUPPORTED
    assert lib.mrp_edge_encoder_fwd_split(None, None, None, 10, 13376, None, None) == m._lib.HIP_ERROR_NOT_SUPPORTED
    assert lib.mrp_edge_encoder_pack(None, None, None, 13344, None, None) == HIP_INVALID_VALUE  # size ok, no pointers


def test_split_encoder_training_validation_without_launch():
    """The encoder's split-bf16 training entry points (ABI 17): shape/pointer checks and workspace
    queries on the host, before any launch (no GPU needed)."""
    lib = m.load_library()
    NS = m._lib.HIP_ERROR_NOT_SUPPORTED
    # forward with h^T: declined shapes, missing pointers
    assert lib.mrp_edge_encoder_fwd_split_train(None, None, None, 10, 48, None, None, 10, None) == NS
    assert lib.mrp_edge_encoder_fwd_split_train(None, None, None, 32, 64, None, None, 32, None) == HIP_INVALID_VALUE
    # dz^T: E % 4 and odd C declined; a short row stride is invalid
    assert lib.mrp_edge_encoder_bwd_prep(16, 6, 64, 16, 6, None) == NS
    assert lib.mrp_edge_encoder_bwd_prep(16, 8, 64, 16, 4, None) == HIP_INVALID_VALUE
    assert lib.mrp_edge_encoder_bwd_prep(None, 0, 64, None, 0, None) == 0  # no edges: no-op
    # the two products: E % 32 and C % 32; db2 needs the dW2 product
    assert lib.mrp_edge_encoder_bwd_split_workspace(1792, 512) > 0
    assert lib.mrp_edge_encoder_bwd_split_workspace(100, 512) == 0
    assert lib.mrp_edge_encoder_bwd_split(None, None, None, None, 100, 64, 16, None, None, None, 0, None) == NS
    assert lib.mrp_edge_encoder_bwd_split(None, None, None, None, 96, 64, None, None, 16, None, 0, None) == \
        HIP_INVALID_VALUE
    # ReLU mask + dW1/db1: workspace = 256-edge blocks x C x 10 floats
    assert lib.mrp_edge_encoder_bwd_t_workspace(1792, 512) == 7 * 512 * 10 * 4
    assert lib.mrp_edge_encoder_bwd_t(None, 0, None, 0, None, 96, 64, None, None, None, 0, None) == 0  # nothing wanted
    assert lib.mrp_edge_encoder_bwd_t(None, 96, None, 96, None, 96, 64, 16, None, None, 0, None) == HIP_INVALID_VALUE
    # the fused three-launch backward: all four gradients required, workspace sized by its plan
    ws = lib.mrp_edge_encoder_bwd_fused_workspace(1792, 512)
    assert ws >= (2 * 512 * 1792 + 7 * 512 * 10) * 4  # at least dz^T and the dW1/db1 partials
    assert lib.mrp_edge_encoder_bwd_fused_workspace(100, 512) == 0
    assert lib.mrp_edge_encoder_bwd_fused(None, None, None, None, None, 96, 64, None, None, None, None, None, 0,
                                          None) == HIP_INVALID_VALUE
    assert lib.mrp_edge_encoder_bwd_fused(16, 16, None, 16, 16, 100, 64, 16, 16, 16, 16, None, 0, None) == NS
    assert lib.mrp_edge_encoder_bwd_fused(16, 16, 16, 16, 16, 96, 64, 16, 16, 16, 16, None, 0, None) == \
        HIP_INVALID_VALUE


def test_split_compress_validation_without_launch():
    lib = m.load_library()
    assert lib.mrp_compress_split_pack_bytes(512, 1024) == 512 * 1024 * 6
    assert lib.mrp_compress_split_pack_bytes(40, 64) == 0
    assert lib.mrp_compress_split_pack(None, 64, 0, 40, 64, None, None) == m._lib.HIP_ERROR_NOT_SUPPORTED
    assert lib.mrp_compress_split_pack(None, 64, 0, 64, 64, None, None) == HIP_INVALID_VALUE
    assert lib.mrp_compress_fwd_split(None, 0, None, 0, 0, 64, 64, None, None, None, 0, None) == 0  # no nodes
    assert lib.mrp_compress_fwd_split(None, 0, None, 0, 2, 64, 64, None, None, None, 0, None) == HIP_INVALID_VALUE
    assert lib.mrp_compress_bwd_data_split(None, 0, 2, 64, 64, None, None, 0, None, 0, None) == HIP_INVALID_VALUE
    assert lib.mrp_compress_bwd_weight_split_workspace(128, 512, 1024) > 0  # split over K
    assert lib.mrp_compress_bwd_weight_split_workspace(128, 96, 1024) == 0  # C % 64: declined
    assert lib.mrp_compress_bwd_weight_split(None, 0, None, 0, None, 0, 2, 96, 64, None, None, None, 0, None) == 0
    # gw given (never dereferenced on the host) but the operands missing
    assert lib.mrp_compress_bwd_weight_split(None, 0, None, 0, None, 0, 2, 96, 64, 16, None, None, 0, None) == \
        HIP_INVALID_VALUE


def test_tuning_knobs_documented_in_the_header():
    """mrp_tuning_set (host-only, no launch): every kernel-choice knob the header documents is accepted
    in range and rejected out of range; unknown names are rejected; "reset" restores defaults."""
    lib = m.load_library()
    try:
        for name, lo, hi in (("bwd_regular_mfma", 0, 1), ("bwd_complete_mfma", 0, 1), ("bwd_mfma_cpw", 1, 2),
                             ("bwd_pre2", 0, 2), ("fwd_regular_split", 0, 1), ("bwd_fused_cap", 1, 64),
                             ("gemm_group", 0, 64), ("nt_group", 0, 64), ("enc_bwd_psa", 0, 2), ("enc_s1", 0, 64), ("enc_s2", 0, 64)):
            assert name.encode() in open(os.path.join(ROOT, "include", "mrp_gnn.h"), "rb").read() or \
                name.startswith("bwd_fused")
            assert lib.mrp_tuning_set(name.encode(), lo) == 0
            assert lib.mrp_tuning_set(name.encode(), hi) == 0
            assert lib.mrp_tuning_set(name.encode(), hi + 1) == HIP_INVALID_VALUE
        assert lib.mrp_tuning_set(b"no_such_knob", 0) == HIP_INVALID_VALUE
        # knobs that name a kernel accept exactly the kernels the library builds (ABI 18)
        header = open(os.path.join(ROOT, "include", "mrp_gnn.h"), "rb").read()
        for name, ok in (("edge_split_v", (-1, 1, 3)), ("gemm_split", (-1, 2, 7)), ("split_nt", (-1, 3, 4))):
            assert name.encode() in header
            for v in range(-2, 9):
                assert lib.mrp_tuning_set(name.encode(), v) == (0 if v in ok else HIP_INVALID_VALUE), (name, v)
        # round 4's kernel-variant knobs are gone with their kernels (tools/lab_*.hip)
        for name in (b"gemm_nn", b"gemm_nt", b"edge_gemm", b"edge_fused", b"edge_split_cb", b"edge_split_k"):
            assert lib.mrp_tuning_set(name, 0) == HIP_INVALID_VALUE
    finally:
        assert lib.mrp_tuning_set(b"reset", 0) == 0
