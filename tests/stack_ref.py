"""Test infrastructure: a plain-torch restatement of the GCN layer stack (any dtype, any device), for
full-size GPU checks where the CPU oracle would take minutes.  Same math as the reference
(``dgl/model/models.py:142-155,180-189,207-211``; residual ``dgl/model/dgl_models.py:36-37``) written
as gather -> FiLM message -> scatter-add -> divide by in-degree, 1x1 convs as matmuls.

Run in float64 it is the accuracy yardstick: a result is accepted when its error against the float64
stack is within max(1e-5, 4 x the error of the same restatement run in float32) — i.e. the HIP path
is as accurate as an fp32 computation of the reference's own op sequence, whatever summation order
the GEMMs (K = C or 2C terms) and the encoder use.
"""
import torch
import torch.nn.functional as F


def edge_gb(params, prefix, pose):
    """``edge_encoder`` (models.py:146-154): (E, C, 2) interleaved sigmoid(gamma, beta)."""
    dt = params[prefix + "layers.0.weight"].dtype
    h = F.relu(F.linear(pose.to(dt), params[prefix + "layers.0.weight"], params[prefix + "layers.0.bias"]))
    z = torch.sigmoid(F.linear(h, params[prefix + "layers.2.weight"], params[prefix + "layers.2.bias"]))
    return z.view(z.shape[0], -1, 2)


def aggregate(x, gb, src, dst):
    """update_all(edge_udf, node_udf) (models.py:207-211,223): mean over in-edges, zeros for in-degree 0."""
    msg = gb[:, :, 0, None, None] * x.index_select(0, src) + gb[:, :, 1, None, None]
    acc = torch.zeros_like(x).index_add_(0, dst, msg)
    deg = torch.bincount(dst, minlength=x.shape[0]).clamp_min(1).to(x.dtype)
    return acc / deg[:, None, None, None]


def conv1x1(h, w, b):
    return torch.einsum("oc,nchw->nohw", w.reshape(w.shape[0], w.shape[1]), h) + b[None, :, None, None]


def stack_forward(params, x, pose, src, dst, layers, combine="cat_compress", alpha=0.1):
    h0 = h = x
    for i in range(1, layers + 1):
        a = aggregate(h, edge_gb(params, f"gcn{i}.edge_encoder.", pose), src, dst)
        if combine == "cat_compress":
            h = conv1x1(torch.cat((h, a), 1), params[f"conv{i}.weight"], params[f"conv{i}.bias"])
        elif combine == "cat":
            h = torch.cat((h, a), 1)
        elif combine == "residual":
            h = h + a
        else:
            h = (1.0 - alpha) * a + alpha * h0
    return h


def run(params, x, pose, src, dst, grad, dtype, loss=None, **kw):
    """(output, dx, {param: grad}) of the restated stack in ``dtype``, backpropagating ``grad``
    (or, with ``loss="square_sum"``, the gradient of ``out.square().sum()``)."""
    p = {k: v.detach().to(dtype).requires_grad_(True) for k, v in params.items()}
    xx = x.detach().to(dtype).requires_grad_(True)
    out = stack_forward(p, xx, pose, src, dst, **kw)
    if loss == "square_sum":
        out.square().sum().backward()
    else:
        out.backward(grad.to(dtype))
    return out.detach(), xx.grad, {k: v.grad for k, v in p.items()}


def err(a, ref):
    a = a.detach().double().cpu()
    ref = ref.detach().double().cpu()
    return float((a - ref).abs().max() / ref.abs().max().clamp_min(1e-300))


def within(ours, f32, f64, floor=1e-5):
    """ours is at least as close to the float64 result as 4x the fp32 restatement (or 1e-5)."""
    e_ours, e_ref = err(ours, f64), err(f32, f64)
    return e_ours <= max(floor, 4.0 * e_ref), (e_ours, e_ref)
