"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's GCN message-passing path, used by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg as the *checker*.
Nothing in the product package (``multi-robot-perception-gnn-1_amd/``) imports it; the product
path has no CPU fallback and fails loudly without its HIP library.

Pinning: the restatement is checked against golden vectors generated in the survey container by
importing the reference's own ``dgl/model/models.py`` (``edge_encoder``, ``edge_udf``,
``node_udf``, ``GCN``) with stub ``dgl``/``torchvision`` modules and driving it through a literal
restatement of DGL's ``update_all`` degree bucketing (``tests/golden/make_golden.py``).  DGL itself
is not installed (third-party, version unpinned by the reference); its bucketing/zero-fill
behaviour is "parity unpinned" beyond that restatement — see DESIGN.md.
"""
from .dgl_udf import (edge_encoder_forward, film_aggregate, film_aggregate_grads, gcn_forward,  # noqa: F401
                      update_all)
from .relpose import cal_relative_pose, quat_to_so3  # noqa: F401
