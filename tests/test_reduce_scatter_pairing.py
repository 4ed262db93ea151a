"""The lane pairing of film_bwd_fused's reduce-scatter (``reduce_scatter64`` / ``rs_step`` in
``csrc/film_mean_kernels.hpp``), simulated on the host: at lane bit b the partner is the xor-32 /
xor-16 lane (ds_bpermute), the row_mirror lane (i <-> 15 - i within 16), the row_half_mirror lane
(i <-> 7 - i within 8) or the quad-perm lane (xor 2, xor 1); a lane whose bit b is set keeps the upper
half of its current range, sends the lower half, and adds what its partner sends.  Steps run from the
group's top lane bit down.  Checked: every lane of every aligned group of L lanes (L = 1..64) ends with
the group sums of exactly the values [gl 64 / L, (gl + 1) 64 / L), gl its index in the group — which
the kernel's stores (lane l stores sum l at L = 64) rely on."""
import numpy as np
import pytest


def partner(lane, bit):
    if bit == 5:
        return lane ^ 32
    if bit == 4:
        return lane ^ 16
    if bit == 3:
        return (lane & ~15) | (15 - (lane & 15))
    if bit == 2:
        return (lane & ~7) | (7 - (lane & 7))
    return lane ^ (2 if bit == 1 else 1)


@pytest.mark.parametrize("L", [1, 2, 4, 8, 16, 32, 64])
def test_reduce_scatter_pairing(L):
    rng = np.random.RandomState(L)
    v = rng.randint(-1000, 1000, size=(64, 64)).astype(np.int64)  # exact integer sums
    orig = v.copy()
    cnt = 64
    for bit in range(L.bit_length() - 2, -1, -1):
        h = cnt // 2
        nv = v.copy()
        for lane in range(64):
            p = partner(lane, bit)
            up, pup = (lane >> bit) & 1, (p >> bit) & 1
            assert up != pup  # partners sit on opposite sides of the bit
            send_p = v[p, :h] if pup else v[p, h:cnt]
            nv[lane, :h] = (v[lane, h:cnt] if up else v[lane, :h]) + send_p
        v, cnt = nv, h
    K = 64 // L
    assert cnt == K
    for lane in range(64):
        gl, g0 = lane % L, lane - lane % L
        want = orig[g0:g0 + L, gl * K:(gl + 1) * K].sum(0)
        assert np.array_equal(v[lane, :K], want), (L, lane)
