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
