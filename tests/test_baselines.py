"""Hand-written baselines (reference lenet5.py / alexnet.py / squeezenet.py)."""
import torch

from featurenet_amd.models.baselines import AlexNet, LeNet5, SqueezeNet, count_params


def test_squeezenet_reference_param_count():
    # squeezenet.py:231 publishes 876,970 params for CIFAR-10 (channels_first quirk)
    assert count_params(SqueezeNet((32, 32, 3), 10, compat=True)) == 876970
    assert count_params(SqueezeNet((32, 32, 3), 10)) == 740554


def test_lenet5_param_count_and_forward():
    m = LeNet5((28, 28, 1), 10)
    assert count_params(m) == 545546        # analytic Keras count of lenet5.py:11-18
    y = m(torch.rand(3, 28, 28, 1))
    assert y.shape == (3, 10)
    y.sum().backward()


def test_squeezenet_alexnet_forward_backward():
    for m, shape in ((SqueezeNet((32, 32, 3), 10, compat=True), (2, 32, 32, 3)),
                     (SqueezeNet((32, 32, 3), 10), (2, 32, 32, 3)),
                     (AlexNet((224, 224, 3), 10), (2, 224, 224, 3))):
        y = m(torch.rand(shape))
        assert y.shape == (2, 10) and torch.isfinite(y).all()
        y.sum().backward()
