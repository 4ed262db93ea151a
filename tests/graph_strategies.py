"""hypothesis strategies for batched robot graphs (shared by tests/test_properties.py and
tests/test_gpu_properties.py): 1-4 graphs of 0-16 nodes, each node 0-max_deg in-edges from any node of
its graph (self-loops and repeated sources allowed), edges of a graph grouped together."""
from hypothesis import strategies as st


@st.composite
def batches(draw, max_graphs=4, max_nodes=16, max_deg=10, min_nodes=0):
    bnn = draw(st.lists(st.integers(min_nodes, max_nodes), min_size=1, max_size=max_graphs))
    src, dst = [], []
    off = 0
    for n in bnn:
        if n:
            edges = []
            for v in range(n):
                k = draw(st.integers(0, max_deg))
                edges += [(draw(st.integers(0, n - 1)), v) for _ in range(k)]
            perm = draw(st.permutations(range(len(edges)))) if edges else []
            for i in perm:
                u, v = edges[i]
                src.append(u + off)
                dst.append(v + off)
        off += n
    return bnn, src, dst
