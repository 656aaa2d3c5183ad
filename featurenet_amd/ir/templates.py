"""Built-in architecture templates.

Reference: ``model/leNet.py:7-40`` (``lenet5_blocks``), ``model/kerasNet.py:7-32``
(``standard_blocks``, the Keras CIFAR-10 example -- including its quirk of
appending block 2's pooling cell to block 1, ``kerasNet.py:24-25``), and the
empty ``model/mobileNet.py`` stub.  ``featurenet3d`` is the north-star voxel
architecture expressed in the same IR (3-D kernels), so it can seed or be
explored by the NAS engine.
"""
from __future__ import annotations

from .spec import BlockSpec, CellSpec, InputSpec, OpSpec


def _conv(kernel, stride, features, padding, act, type="normal"):
    return InputSpec("convolution", kernel=tuple(kernel), stride=None if stride is None else tuple(stride),
                     features=features, padding="same", activation=act, type=type,
                     custom={} if padding == "same" else {"padding": "same"})


def _pool(kernel, stride, type, padding):
    return InputSpec("pooling", kernel=(min(kernel[0], 3), min(kernel[1], 3)),
                     stride=None if stride is None else tuple(stride), padding="same", activation=None, type=type)


def lenet5_blocks() -> list[BlockSpec]:
    b1 = BlockSpec()
    b1.set_stride("1x1")
    b1.set_features(600)
    b1.cells = [CellSpec(input1=_conv((5, 5), None, None, "same", "tanh")),
                CellSpec(input1=_pool((2, 2), None, "average", "valid"))]
    b2 = BlockSpec()
    b2.set_stride("1x1")
    b2.cells = [CellSpec(input1=_conv((5, 5), None, 12, "same", "tanh"))]
    b22 = BlockSpec()
    b22.set_stride("2x2")
    b22.cells = [CellSpec(input1=_pool((2, 2), None, "average", "valid"))]
    b3 = BlockSpec()
    b3.set_stride("1x1")
    b3.cells = [CellSpec(input1=_conv((5, 5), (1, 1), 120, "valid", "tanh"))]
    b4 = BlockSpec()
    b4.set_stride("1x1")
    b4.cells = [CellSpec(input1=InputSpec.dense(84, "tanh"))]
    return [b1, b2, b22, b3, b4]


def standard_blocks() -> list[BlockSpec]:
    # Drop(0.25) in the reference is int(0.25)/100 == 0 -> no dropout (kept).
    drop = OpSpec("dropout", value=0.0)
    b1 = BlockSpec()
    b1.cells = [CellSpec(input1=_conv((3, 3), (1, 1), 32, "same", "relu")),
                CellSpec(input1=_conv((3, 3), (1, 1), 32, "same", "relu")),
                CellSpec(input1=_pool((2, 2), (1, 1), "max", "valid"), op1=OpSpec("dropout", value=0.0))]
    b2 = BlockSpec()
    b2.cells = [CellSpec(input1=_conv((3, 3), (1, 1), 64, "same", "relu")),
                CellSpec(input1=_conv((3, 3), (1, 1), 64, "same", "relu"))]
    b1.cells.append(CellSpec(input1=_pool((2, 2), (1, 1), "max", "valid"), op1=drop))
    b4 = BlockSpec()
    b4.cells = [CellSpec(input1=InputSpec.dense(512, "relu"), op1=OpSpec("dropout", value=0.0))]
    return [b1, b2, b4]


def mobilenet_blocks() -> list[BlockSpec]:
    return []   # the reference stub is empty and never wired


def featurenet3d_blocks() -> list[BlockSpec]:
    """FeatureNet-3D convolution stack as IR blocks (3-D kernels, valid-equivalent strides)."""
    blocks = []
    for k, s, f, bn in ((7, 2, 32, True), (5, 1, 32, True), (4, 1, 64, True), (3, 1, 64, True)):
        c = CellSpec(input1=InputSpec("convolution", kernel=(k, k, k), stride=(s, s, s), features=f,
                                      padding="valid", activation=None, type="normal"),
                     op1=OpSpec("batchnorm", axis=-1))
        c2 = CellSpec(input1=InputSpec.identity(), op1=OpSpec("activation", method="relu"))
        blocks.append(BlockSpec(cells=[c, c2]))
    blocks.append(BlockSpec(cells=[CellSpec(input1=InputSpec("pooling", kernel=(2, 2, 2), stride=(2, 2, 2),
                                                             padding="valid", activation=None, type="max"),
                                            op1=OpSpec("flatten"))]))
    blocks.append(BlockSpec(cells=[CellSpec(input1=InputSpec.dense(128, "relu"))]))
    return blocks


TEMPLATES = {
    "lenet5": lenet5_blocks,
    "keras": standard_blocks,
    "mobilenet": mobilenet_blocks,
    "featurenet3d": featurenet3d_blocks,
}


def get_template(name: str) -> list[BlockSpec]:
    fn = TEMPLATES.get(name)
    return fn() if fn else []
