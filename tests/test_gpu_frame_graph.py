"""GPU: per-frame graphs built on the device (``mrp_frame_graph_build`` via ``frame_batch``) against
the host builders (``frame_graph`` + ``batch``), which are pinned to the reference's own relative
poses (``tests/golden/relpose.npz``).  Everything here is integer or reproduces the reference's
float32 expression order, so the bar is bit-exact."""
import numpy as np
import pytest
import torch

import mrp_gnn_amd as m
from conftest import load_golden

pytestmark = pytest.mark.gpu


def random_poses(rng, B, n, spread=10.0):
    t = rng.uniform(-spread, spread, size=(B, n, 3))
    q = rng.standard_normal((B, n, 4))
    q /= np.linalg.norm(q, axis=-1, keepdims=True)
    return np.concatenate([t, q], -1).astype(np.float32)


def host_batch(poses, knn=None):
    return m.batch([m.frame_graph(p, knn=knn) for p in poses])


def assert_same_graph(gd, gh, dev):
    sd, dd = (t.numpy() for t in gd.edges())
    sh, dh = (t.numpy() for t in gh.edges())
    assert np.array_equal(sd, sh) and np.array_equal(dd, dh)
    pd, ph = gd.edata["pose"].cpu().numpy(), gh.edata["pose"].numpy()
    assert pd.dtype == ph.dtype == np.float32
    assert np.array_equal(pd, ph), f"max abs diff {np.abs(pd - ph).max()}"
    assert gd.batch_num_nodes().tolist() == gh.batch_num_nodes().tolist()
    assert gd.batch_num_edges().tolist() == gh.batch_num_edges().tolist()
    cd = gd.csr(dev)
    ch = gh.csr(dev)
    assert cd.graph_kind == ch.graph_kind and cd.max_nodes == ch.max_nodes
    for a in ("indptr", "src", "eid", "graph_off"):
        if cd.graph_kind == m._lib.GRAPH_COMPLETE and a != "graph_off":
            # not read by the kernels for complete graphs, but the device builder writes them anyway
            pass
        assert torch.equal(getattr(cd, a).cpu(), getattr(ch, a).cpu()), a


def test_relpose_bitexact_against_reference_fixture(cuda_device):
    z = load_golden("relpose")
    poses = np.stack([z["p1"], z["p2"]], 1)  # 64 frames of 2 robots: edge 0->1 = cal_relative_pose(p1, p2)
    g = m.frame_batch(torch.from_numpy(poses).to(cuda_device))
    rel = g.edata["pose"].cpu().numpy().reshape(-1, 2, 9)
    assert np.array_equal(rel[:, 0], z["out"])
    assert np.array_equal(rel[:, 1], m.relative_pose_batch(z["p2"], z["p1"]))


@pytest.mark.parametrize("n", list(range(1, 17)))
def test_complete_matches_host(cuda_device, n):
    rng = np.random.RandomState(n)
    poses = random_poses(rng, 5, n)
    gd = m.frame_batch(torch.from_numpy(poses).to(cuda_device))
    gh = host_batch(poses)
    assert gd.is_complete() and gh.is_complete()
    assert_same_graph(gd, gh, cuda_device)
    csr = gh.host_csr()
    got = gd.csr(cuda_device, allow_complete=False, allow_regular=False)
    for a, b in zip(("indptr", "src", "eid", "graph_off"), csr[:4]):
        assert np.array_equal(getattr(got, a).cpu().numpy(), b), a


@pytest.mark.parametrize("n,k", [(2, 1), (5, 2), (8, 4), (9, 4), (12, 7), (16, 4), (16, 8), (16, 15)])
def test_knn_matches_host(cuda_device, n, k):
    rng = np.random.RandomState(100 * n + k)
    poses = random_poses(rng, 6, n)
    gd = m.frame_batch(torch.from_numpy(poses).to(cuda_device), knn=k)
    gh = host_batch(poses, knn=k)
    assert gd.in_degree_k() == gh.in_degree_k() == k
    assert_same_graph(gd, gh, cuda_device)


def test_knn_ties_go_to_lower_index(cuda_device):
    # robots on a small integer lattice and repeated positions: many equal distances
    rng = np.random.RandomState(7)
    B, n = 8, 12
    poses = random_poses(rng, B, n)
    poses[..., :3] = rng.randint(-1, 2, size=(B, n, 3)).astype(np.float32)
    poses[0, :, :3] = 0.0  # all robots at one point: every distance is 0
    for k in (1, 3, 6, 11):
        gd = m.frame_batch(torch.from_numpy(poses).to(cuda_device), knn=k)
        gh = host_batch(poses, knn=k)
        assert_same_graph(gd, gh, cuda_device)
    src = m.frame_batch(torch.from_numpy(poses[:1]).to(cuda_device), knn=3).edges()[0].numpy()
    assert src.reshape(n, 3).tolist() == [[u for u in range(n) if u != v][:3] for v in range(n)]


def test_device_graph_drives_the_aggregation(cuda_device):
    """A GCN layer over a device-built batch equals the same layer over the host-built batch."""
    import types
    rng = np.random.RandomState(3)
    for knn in (None, 4):
        poses = random_poses(rng, 4, 9)
        gd = m.frame_batch(torch.from_numpy(poses).to(cuda_device), knn=knn)
        gh = host_batch(poses, knn=knn).to(cuda_device)
        torch.manual_seed(0)
        gcn = m.GCN(types.SimpleNamespace(feature_dim=16)).to(cuda_device)
        x = torch.randn(gd.num_nodes(), 16, 8, 8, device=cuda_device)
        gd.ndata["image"] = x
        gh.ndata["image"] = x
        assert torch.equal(gcn(gd), gcn(gh))


def test_empty_and_invalid(cuda_device):
    g = m.frame_batch(torch.zeros(0, 4, 7, device=cuda_device))
    assert g.num_nodes() == 0 and g.num_edges() == 0
    g = m.frame_batch(torch.zeros(3, 1, 7, device=cuda_device))  # single robots: no edges
    assert g.num_nodes() == 3 and g.num_edges() == 0
    with pytest.raises(ValueError):
        m.frame_batch(torch.zeros(2, 17, 7, device=cuda_device))
    with pytest.raises(ValueError):
        m.frame_batch(torch.zeros(2, 4, 7, device=cuda_device), knn=4)
    with pytest.raises(ValueError):
        m.frame_batch(torch.zeros(2, 4, 6, device=cuda_device))
