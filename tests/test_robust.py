"""Robustness: attacks move predictions, perturbation budgets hold, CLEVER is sane.

Parity with the reference's ART/cleverhans numbers is unpinned (neither library
is importable here); the checks are the defining properties of each method.
"""
import math

import numpy as np
import pytest
import torch

from featurenet_amd.robust import attacks as A
from featurenet_amd.robust.evaluate import eval_robustness
from featurenet_amd.robust.metrics import clever_u, random_sphere


class _Lin(torch.nn.Module):
    """Linear 2-class model on 4-d inputs: margins and gradients known in closed form."""

    def __init__(self):
        super().__init__()
        self.fc = torch.nn.Linear(4, 2)
        with torch.no_grad():
            self.fc.weight.copy_(torch.tensor([[1.0, 0, 0, 0], [-1.0, 0, 0, 0]]))
            self.fc.bias.zero_()

    def forward(self, x):
        return self.fc(x.reshape(len(x), -1))


def _data():
    x = torch.tensor([[0.3, 0.1, 0.2, 0.0], [-0.4, 0.5, 0.0, 0.1], [0.2, 0.0, 0.0, 0.0]])
    y = (x[:, 0] < 0).long()
    return x, y


def test_fgsm_linf_budget_and_flip():
    m = _Lin()
    x, y = _data()
    adv = A.fgsm(m, x, y, eps=0.5, norm=float("inf"), clip=None)
    assert torch.all((adv - x).abs() <= 0.5 + 1e-6)
    assert torch.all(A.predict(m, adv).argmax(-1) != y)


def test_pgd_l2_projection():
    m = _Lin()
    x, y = _data()
    adv = A.pgd(m, x, y, eps=0.25, eps_step=0.1, norm=2, clip=None)
    assert torch.all((adv - x).flatten(1).norm(dim=1) <= 0.25 + 1e-5)
    # samples with margin < eps flip (|x0| * 2 margin over sqrt(2)-scaled logit gap)
    assert A.predict(m, adv).argmax(-1)[2] != y[2]


def test_carlini_l2_finds_minimal_perturbation():
    m = _Lin()
    x, y = _data()
    adv = A.carlini_l2(m, x, y, max_iter=200, binary_search_steps=6, learning_rate=0.05, clip=None)
    flipped = A.predict(m, adv).argmax(-1) != y
    assert flipped.all()
    # minimal L2 distance to the decision boundary x0 = 0 is |x0|
    dist = (adv - x).flatten(1).norm(dim=1)
    assert torch.all(dist <= x[:, 0].abs() * 1.5 + 0.05)


def test_random_sphere_norms():
    rng = np.random.default_rng(0)
    p2 = random_sphere(200, 5, 2.0, 2, rng)
    assert np.all(np.linalg.norm(p2, axis=1) <= 2.0 + 1e-9)
    pinf = random_sphere(200, 5, 0.3, np.inf, rng)
    assert np.all(np.abs(pinf) <= 0.3 + 1e-9)


def test_clever_linear_model():
    """For a linear model the local Lipschitz constant of the margin is exact:
    CLEVER ~= margin / ||w0 - w1||_2 = |x0| * 2 / 2."""
    m = _Lin()
    x, _ = _data()
    s = clever_u(m, x[0], nb_batches=10, batch_size=20, radius=2.0, norm=2, pool_factor=3, clip=None)
    assert s == pytest.approx(abs(float(x[0, 0])) * 2 / 2.0, rel=0.1)


def test_eval_robustness_policy():
    m = _Lin()
    x, y = _data()
    out = eval_robustness(m, (x, y), ["fgsm", "pgd"], set_size=3, clip=(-5.0, 5.0))
    assert set(out) >= {"fgsm", "pgd", "score", "time_s"}
    score, clean, adv = out["pgd"]
    assert clean == 1.0 and adv <= clean and math.isfinite(score)
    assert out["score"] == out["fgsm"][0]
    assert eval_robustness(m, (x, y), ["fgsm"], accuracy=0.4)["skipped"]


def test_native_weibull_fit_matches_scipy():
    """csrc/runtime/weibull.cpp runs scipy's estimator (weibull_min.fit with a shape guess,
    optimizer fmin) step for step: same parameters on random CLEVER-like problems."""
    from scipy.stats import weibull_min

    from featurenet_amd import _native
    from featurenet_amd.robust.metrics import _fmin, weibull_locs

    rng = np.random.default_rng(1)
    maxes = np.stack([rng.random(10) * rng.uniform(0.05, 5) + rng.uniform(0, 3) for _ in range(40)])
    ref = np.array([weibull_min.fit(-m, 1.0, optimizer=_fmin) for m in maxes])
    if _native.runtime_available():
        fit = _native.runtime().weibull_min_fit_batch(-maxes, 1.0, 1e-6, 1e-4, 1000, 2)
        np.testing.assert_allclose(fit, ref, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(weibull_locs(maxes, 1.0), ref[:, 1], rtol=1e-9, atol=1e-12)


class _Small(torch.nn.Module):
    """A nonlinear 3-class model on 2x3x3x1 inputs (class gradients vary over the pool)."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        self.w1 = torch.nn.Parameter(torch.randn(18, 8, generator=g))
        self.w2 = torch.nn.Parameter(torch.randn(8, 3, generator=g))

    def forward(self, x):
        return torch.tanh(x.reshape(len(x), -1) @ self.w1) @ self.w2


def test_clever_batch_equals_per_sample_reference_loop():
    """The batched CLEVER gives the reference's literal loop exactly: for each sample, for each
    target class, a fresh pool and fresh batch draws from ONE generator advanced in the
    reference's order (``model/metrics.py:284-302`` under ``tensorflow_generator.py:200-201``),
    with the default generator and with the legacy ``np.random`` stream (RandomState)."""
    from featurenet_amd.robust.metrics import clever_batch, clever_t_literal, clever_u_batch

    m = _Small()
    xs = torch.rand(7, 2, 3, 3, 1, generator=torch.Generator().manual_seed(2))
    preds = A.predict(m, xs).argmax(-1).tolist()
    for mk in (lambda: np.random.default_rng(0), lambda: np.random.RandomState(5)):
        batched = clever_batch(m, xs, nb_batches=10, batch_size=5, radius=2.0, norm=2, pool_factor=3,
                               clip=(0.0, 1.0), rng=mk(), chunk_points=30)      # 2 problems per chunk
        rng = mk()
        for i in range(len(xs)):
            tg = [j for j in range(3) if j != preds[i]]
            assert sorted(batched[i]) == tg
            for j in tg:
                ref = clever_t_literal(m, xs[i], j, 10, 5, 2.0, 2, 1.0, 3, (0.0, 1.0), rng)
                assert batched[i][j] == pytest.approx(ref, rel=1e-5, abs=1e-7)
    u = clever_u_batch(m, xs, 10, 5, 2.0, 2, pool_factor=3, clip=(0.0, 1.0))
    again = clever_batch(m, xs, 10, 5, 2.0, 2, pool_factor=3, clip=(0.0, 1.0))
    assert u == pytest.approx([min(d.values()) for d in again])


class _CountingRng:
    """A generator wrapper that records the pool draws (their first values)."""

    def __init__(self, seed):
        self.g, self.pools, self.choices = np.random.default_rng(seed), [], 0

    def standard_normal(self, shape):
        a = self.g.standard_normal(shape)
        self.pools.append(a[0, 0])
        return a

    def choice(self, n, k):
        self.choices += 1
        return self.g.choice(n, k)


def test_clever_pools_are_distinct_per_sample_and_target():
    """Every (sample, target) problem draws its own pool and its own nb_batches index batches
    (round 4 shared one seed-0 pool and one draw table across all problems)."""
    from featurenet_amd.robust.metrics import clever_batch

    m = _Small()
    xs = torch.rand(4, 2, 3, 3, 1, generator=torch.Generator().manual_seed(3))
    rng = _CountingRng(1)
    out = clever_batch(m, xs, nb_batches=10, batch_size=5, radius=2.0, norm=2, pool_factor=3, rng=rng)
    q = sum(len(d) for d in out)
    assert q == 4 * 2
    assert len(rng.pools) == q and len(set(rng.pools)) == q
    assert rng.choices == q * 10


def test_attacks_take_no_parameter_gradients():
    """Input gradients only: parameters end with requires_grad restored and no .grad written
    (on the GPU the same switch keeps every weight-gradient kernel from launching)."""
    m = _Small()
    x = torch.rand(4, 2, 3, 3, 1)
    y = torch.tensor([0, 1, 2, 0])
    g = A.loss_gradient(m, x, y)
    assert g.shape == x.shape and torch.isfinite(g).all()
    cg = A.class_gradients(m, x, max_rows=6)                       # 2 chunks of 2 samples x 3 classes
    full = A.class_gradients(m, x)
    torch.testing.assert_close(cg, full)
    A.carlini_l2(m, x, y, binary_search_steps=2, max_iter=3)
    A.pgd(m, x, y, max_iter=3)
    assert all(p.requires_grad and p.grad is None for p in m.parameters())
