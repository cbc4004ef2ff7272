"""Numerics of the ltorch decompositions in ``torch/more_ops.py`` against eager PyTorch (fp64,
forward and gradients), plus a check that each op shows up in the trace as its own symbol."""
import pytest
import torch

import lightning_thunder_amd as lta

F = torch.nn.functional

# each case: fn(x, y, p, W, z) with x,y [4,6] normal, p [4,6] in (0,1), W [3,6,5], z [4,5]
CASES = {
    "smooth_l1_loss": lambda x, y, p, W, z: F.smooth_l1_loss(x, y, beta=0.7),
    "huber_loss": lambda x, y, p, W, z: F.huber_loss(x, y, delta=0.5),
    "binary_cross_entropy": lambda x, y, p, W, z: F.binary_cross_entropy(p, (y > 0).double()),
    "kl_div": lambda x, y, p, W, z: F.kl_div(x.log_softmax(-1), p, reduction="batchmean"),
    "kl_div_log_target": lambda x, y, p, W, z: F.kl_div(x.log_softmax(-1), y.log_softmax(-1), reduction="sum",
                                                        log_target=True),
    "poisson_nll_loss": lambda x, y, p, W, z: F.poisson_nll_loss(x, p * 3, full=True),
    "soft_margin_loss": lambda x, y, p, W, z: F.soft_margin_loss(x, y.sign().detach()),
    "cosine_similarity": lambda x, y, p, W, z: F.cosine_similarity(x, y),
    "pairwise_distance": lambda x, y, p, W, z: F.pairwise_distance(x, y),
    "pairwise_distance_p3": lambda x, y, p, W, z: F.pairwise_distance(x, y, p=3.0, keepdim=True),
    "triplet_margin_loss": lambda x, y, p, W, z: F.triplet_margin_loss(x, y, p, swap=True),
    "cosine_embedding_loss": lambda x, y, p, W, z: F.cosine_embedding_loss(x, y, (z[:, 0] > 0).double() * 2 - 1),
    "gaussian_nll_loss": lambda x, y, p, W, z: F.gaussian_nll_loss(x, y, p + 0.1, full=True),
    "multilabel_soft_margin_loss": lambda x, y, p, W, z: F.multilabel_soft_margin_loss(x, (y > 0).double()),
    "hinge_embedding_loss": lambda x, y, p, W, z: F.hinge_embedding_loss(x, y.sign()),
    "margin_ranking_loss": lambda x, y, p, W, z: F.margin_ranking_loss(x, y, z[:, :1].sign().expand(4, 6), margin=0.1),
    "logaddexp": lambda x, y, p, W, z: torch.logaddexp(x, y),
    "logaddexp2": lambda x, y, p, W, z: torch.logaddexp2(x, y),
    "xlogy": lambda x, y, p, W, z: torch.xlogy(x, p),
    "xlog1py": lambda x, y, p, W, z: torch.special.xlog1py(x, p),
    "hypot": lambda x, y, p, W, z: torch.hypot(x, y),
    "logit": lambda x, y, p, W, z: torch.logit(p, 1e-3),
    "sinc": lambda x, y, p, W, z: torch.sinc(x),
    "deg2rad": lambda x, y, p, W, z: torch.deg2rad(x),
    "frac": lambda x, y, p, W, z: torch.frac(x * 3),
    "fmax": lambda x, y, p, W, z: torch.fmax(x, y),
    "fmin": lambda x, y, p, W, z: torch.fmin(x, y),
    "float_power": lambda x, y, p, W, z: torch.float_power(p, 2.5),
    "erfcx": lambda x, y, p, W, z: torch.special.erfcx(p),
    "nansum": lambda x, y, p, W, z: torch.nansum(x, 1),
    "nanmean": lambda x, y, p, W, z: torch.nanmean(x, 0),
    "cumprod": lambda x, y, p, W, z: torch.cumprod(x, 1),
    "logcumsumexp": lambda x, y, p, W, z: torch.logcumsumexp(x, 1),
    "diff": lambda x, y, p, W, z: torch.diff(x, n=2, dim=1),
    "diff_prepend": lambda x, y, p, W, z: torch.diff(x, dim=0, prepend=y[:1]),
    "trace": lambda x, y, p, W, z: torch.trace(x),
    "dot": lambda x, y, p, W, z: torch.dot(x[0], y[0]),
    "vdot": lambda x, y, p, W, z: torch.vdot(x[1], y[2]),
    "inner": lambda x, y, p, W, z: torch.inner(x, y),
    "mv": lambda x, y, p, W, z: torch.mv(x, y[0]),
    "addmv": lambda x, y, p, W, z: torch.addmv(x[:, 0], x, y[0], beta=0.5, alpha=2),
    "addr": lambda x, y, p, W, z: torch.addr(x, x[:, 0], y[0], beta=0.5, alpha=2),
    "addbmm": lambda x, y, p, W, z: torch.addbmm(z, W.transpose(1, 2)[:, :4, :], W[:, :, :5], beta=0.5),
    "kron": lambda x, y, p, W, z: torch.kron(x, y[:2, :3]),
    "tensordot": lambda x, y, p, W, z: torch.tensordot(x, y, dims=([1], [1])),
    "tensordot_int": lambda x, y, p, W, z: torch.tensordot(x, W.transpose(0, 1), dims=1),
    "bilinear": lambda x, y, p, W, z: F.bilinear(x, z, W, z[0, :3]),
    "dstack": lambda x, y, p, W, z: torch.dstack([x, y]),
    "column_stack": lambda x, y, p, W, z: torch.column_stack([x[:, 0], y]),
    "hsplit": lambda x, y, p, W, z: torch.hsplit(x, 3),
    "vsplit": lambda x, y, p, W, z: torch.vsplit(x, [1, 3]),
    "broadcast_tensors": lambda x, y, p, W, z: torch.broadcast_tensors(x[:1], y),
    "pixel_shuffle": lambda x, y, p, W, z: F.pixel_shuffle(x.reshape(1, 4, 2, 3), 2),
    "pixel_unshuffle": lambda x, y, p, W, z: F.pixel_unshuffle(x.reshape(1, 1, 4, 6), 2),
    "rot90_1": lambda x, y, p, W, z: torch.rot90(x, 1),
    "rot90_2": lambda x, y, p, W, z: torch.rot90(x, 2),
    "rot90_3": lambda x, y, p, W, z: torch.rot90(x, 3),
    "tile": lambda x, y, p, W, z: torch.tile(x, (2,)),
    "block_diag": lambda x, y, p, W, z: torch.block_diag(x, y[:2, :3]),
    "cartesian_prod": lambda x, y, p, W, z: torch.cartesian_prod(x[0, :2], y[0, :3]),
    "meshgrid_xy": lambda x, y, p, W, z: torch.meshgrid(x[0], y[1, :3], indexing="xy"),
    "eye": lambda x, y, p, W, z: torch.eye(4, 6, dtype=torch.float64) * x,
}
# ops without a gradient through the compared output
NONDIFF = {
    "heaviside": lambda x, y, p, W, z: torch.heaviside(x.round(), y),
    "vander": lambda x, y, p, W, z: torch.vander(x[0], 4),  # eager vander has no usable backward
    "isclose": lambda x, y, p, W, z: torch.isclose(x, x + 1e-9),
    "count_nonzero": lambda x, y, p, W, z: torch.count_nonzero(x.round(), 0),
    "isposinf": lambda x, y, p, W, z: torch.isposinf(x / (x.round())),
    "isneginf": lambda x, y, p, W, z: torch.isneginf(x / (x.round())),
}


def _inputs():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 6, dtype=torch.float64, generator=g)
    y = torch.randn(4, 6, dtype=torch.float64, generator=g)
    p = torch.rand(4, 6, dtype=torch.float64, generator=g) * 0.9 + 0.05
    W = torch.randn(3, 6, 5, dtype=torch.float64, generator=g)
    z = torch.randn(4, 5, dtype=torch.float64, generator=g)
    return x, y, p, W, z


def _flat(o):
    return list(o) if isinstance(o, (tuple, list)) else [o]


@pytest.mark.parametrize("name", sorted(CASES))
def test_more_ops_fwd_bwd(name):
    fn = CASES[name]
    ins = _inputs()
    ref_in = [t.clone().requires_grad_() for t in ins]
    ours_in = [t.clone().requires_grad_() for t in ins]
    ref = _flat(fn(*ref_in))
    jf = lta.jit(fn)
    out = _flat(jf(*ours_in))
    assert len(ref) == len(out)
    for r, o in zip(ref, out):
        torch.testing.assert_close(o, r)
    # gradients of a weighted sum of all outputs
    g = torch.Generator().manual_seed(1)
    ws = [torch.randn(r.shape, dtype=r.dtype, generator=g) for r in ref]
    rl = sum((r * w).sum() for r, w in zip(ref, ws))
    ol = sum((o * w).sum() for o, w in zip(out, ws))
    used = [i for i, t in enumerate(ref_in) if torch.autograd.grad(rl, t, retain_graph=True, allow_unused=True)[0] is not None]
    if not used:
        return
    rg = torch.autograd.grad(rl, [ref_in[i] for i in used])
    og = torch.autograd.grad(ol, [ours_in[i] for i in used], allow_unused=True)
    for r, o in zip(rg, og):
        torch.testing.assert_close(o if o is not None else torch.zeros_like(r), r)


@pytest.mark.parametrize("name", sorted(NONDIFF))
def test_more_ops_nondiff(name):
    ins = _inputs()
    torch.testing.assert_close(lta.jit(NONDIFF[name])(*ins), NONDIFF[name](*ins))


@pytest.mark.parametrize("name,sym", [("smooth_l1_loss", "smooth_l1_loss"), ("logaddexp", "logaddexp"),
                                      ("kron", "kron"), ("cumprod", "cumprod"), ("tensordot", "tensordot")])
def test_more_ops_are_symbols(name, sym):
    ins = _inputs()
    jf = lta.jit(CASES[name])
    jf(*ins)
    assert sym in str(lta.last_traces(jf)[0])


def test_more_ops_cumprod_zeros_and_signs():
    x = torch.tensor([[2.0, -1.0, 0.0, 3.0], [-2.0, -0.5, 4.0, 1.0]], dtype=torch.float64)
    torch.testing.assert_close(lta.jit(lambda t: torch.cumprod(t, 1))(x), torch.cumprod(x, 1))


@pytest.mark.parametrize("name,args,stat,expected,tol", [
    ("normal_", (2.0, 3.0), "mean", 2.0, 0.05), ("normal_", (2.0, 3.0), "std", 3.0, 0.05),
    ("log_normal_", (0.0, 0.5), "mean", 1.1331, 0.02), ("exponential_", (2.0,), "mean", 0.5, 0.01),
    ("cauchy_", (), "median", 0.0, 0.02), ("geometric_", (0.3,), "mean", 1 / 0.3, 0.05),
    ("random_", (3, 10), "mean", 6.0, 0.05),
])
def test_more_ops_inplace_samplers(name, args, stat, expected, tol):
    x = torch.zeros(200000)
    r = lta.jit(lambda t: getattr(t.clone(), name)(*args))(x)
    assert r.shape == x.shape
    assert abs(getattr(r, stat)().item() - expected) < tol
    if name == "random_":
        assert r.min().item() >= 3 and r.max().item() <= 9 and torch.equal(r, r.floor())
