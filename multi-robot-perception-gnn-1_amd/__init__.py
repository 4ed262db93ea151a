"""MI355X-native (gfx950) GCN message passing for multi-robot perception.

Drop-in replacement for the DGL FiLM-mean GCN hot path of xjh19971/multi-robot-perception-gnn-1
(``dgl/model/models.py:142-226``): a DGL-free batched graph, the reference's model classes with
identical ``state_dict`` keys, and hand-written HIP kernels behind the C ABI in
``include/mrp_gnn.h``.  Import as ``mrp_gnn_amd`` (the repo-root alias module; this directory's
name is not a Python identifier).
"""
from ._lib import MAX_NODES, MAX_REGULAR_K, MODES, graph_regular, load_library  # noqa: F401
from .aggregate import (EpilogueSpec, FilmMeanFunction, film_mean, film_mean_cat,  # noqa: F401
                        film_mean_cat_forward_into, film_mean_forward_into, film_mean_mix, film_mean_residual)
from . import compat, compress, encoder  # noqa: F401
from .device_graph import frame_batch  # noqa: F401
from .graph import (GraphCSR, RobotGraph, batch, complete_edges, complete_graph, frame_graph,  # noqa: F401
                    graph, knn_edges, load_graphs, save_graphs, unbatch)
from .models import (GCN, GCNBlock, GCNStack, clear_packed_weights, edge_encoder, multi_view_dgl_model,  # noqa: F401
                     stack_layout)
from .pose import cal_relative_pose, quat_to_so3, relative_pose_batch  # noqa: F401

__version__ = "0.1.0"
