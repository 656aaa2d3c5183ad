"""Typed run configuration (replaces the reference's class-attribute globals).

The reference configures a search through mutable class attributes
(``MutableBase.MAX_NB_CELLS``, ``mutation_stategy``, ``selection_strategy``,
``TensorflowGenerator.default_batchsize`` ... -- SURVEY 5.6) and a getopt CLI
(``run.py:49-104``).  Here one dataclass holds everything, loadable from
YAML/JSON and overridable from the command line (:mod:`featurenet_amd.cli`),
with the reference flag names kept as aliases.  Reference CLI bugs are not
reproduced: ``--fpath`` sets the feature model (it overwrote the base path,
``run.py:72-73``), ``--selection_strategy`` takes effect (it set an unused
attribute, ``run.py:89-93``) and ``--nb BxCxN`` is honoured (the meta model was
hard-coded to 5x5x100, ``run.py:116``).
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field, fields
from pathlib import Path


@dataclass
class SearchConfig:
    nb: str = "10x5x100"                 # BLOCKSxCELLSxPRODUCTS, or just PRODUCTS
    training_epochs: int = 5
    base_path: str = "./products"
    fm_path: str = ""                    # 1-block template ("" = built-in search space)
    pledge_duration: float = 30.0
    products_file: str = ""              # existing .pdt to start from
    dataset: str = "mnist"
    mutation_strategy: str = "random"    # random (= CHOICE) | all
    selection_strategy: str = "pareto"   # pareto | elitist | hybrid
    mutation_rate: float = 0.1
    survival_rate: float = 0.2
    evolution_epochs: int = 0
    breed: bool = True
    model: str = ""                      # template seed when no products are given
    max_nb_cells: int = 5
    max_nb_blocks: int = 10
    attacks: list = field(default_factory=lambda: ["cw", "pgd"])
    batch_size: int = 64
    devices: str = ""                    # "" = every visible GPU (or cpu); "0,1" / "cpu"
    trial_timeout_s: float = 0.0         # 0 = no watchdog
    workers_per_device: int = 0          # trial worker processes per GPU; 0 = auto (4 per GPU, 1 on the CPU)
    seed: int = 0
    synthetic_sizes: list = field(default_factory=lambda: [6000, 1000])   # when a dataset is not on disk

    @property
    def nb_tuple(self) -> tuple:
        return tuple(int(v) for v in str(self.nb).lower().split("x"))

    def to_dict(self) -> dict:
        return asdict(self)

    @staticmethod
    def load(path: str | Path) -> "SearchConfig":
        text = Path(path).read_text()
        if str(path).endswith((".yaml", ".yml")):
            import yaml

            d = yaml.safe_load(text) or {}
        else:
            d = json.loads(text)
        return SearchConfig.from_dict(d)

    @staticmethod
    def from_dict(d: dict) -> "SearchConfig":
        names = {f.name for f in fields(SearchConfig)}
        unknown = set(d) - names
        if unknown:
            raise ValueError(f"unknown config keys: {sorted(unknown)}")
        return SearchConfig(**d)
