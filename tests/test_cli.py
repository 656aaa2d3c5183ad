"""Command line front-end (reference run.py / pledge_evolution.py / full.py flags)."""
import json
import os

import pytest

from featurenet_amd import _native
from featurenet_amd.cli import build_parser, main
from featurenet_amd.config import SearchConfig

need_rt = pytest.mark.skipif(not _native.runtime_available(), reason="native runtime not built")


def test_reference_flags_parse():
    a = build_parser().parse_args(["run", "-n", "2x3x8", "-t", "2", "-b", "/tmp/x", "-f", "fm.xml", "-i", "5",
                                   "-d", "cifar", "-m", "all", "-g", "elitist", "-r", "0.2", "-s", "0.3",
                                   "-e", "4", "-y", "1", "-l", "lenet5"])
    assert (a.nb, a.training_epochs, a.base_path, a.fm_path, a.pledge_duration) == ("2x3x8", 2, "/tmp/x", "fm.xml", 5)
    assert (a.dataset, a.mutation_strategy, a.selection_strategy) == ("cifar", "all", "elitist")
    assert (a.mutation_rate, a.survival_rate, a.evolution_epochs, a.model) == (0.2, 0.3, 4, "lenet5")


def test_config_file_roundtrip(tmp_path):
    c = SearchConfig(nb="1x1x4", dataset="cifar")
    p = tmp_path / "c.json"
    p.write_text(json.dumps(c.to_dict()))
    assert SearchConfig.load(p) == c
    (tmp_path / "c.yaml").write_text("nb: 2x2x6\nmutation_rate: 0.5\n")
    y = SearchConfig.load(tmp_path / "c.yaml")
    assert y.nb_tuple == (2, 2, 6) and y.mutation_rate == 0.5
    with pytest.raises(ValueError):
        SearchConfig.from_dict({"bogus": 1})


@need_rt
def test_template_extend_sample(tmp_path, capsys):
    t = tmp_path / "tpl.xml"
    assert main(["template", str(t)]) == 0
    out = tmp_path / "nas_2_2.xml"
    assert main(["extend", "--input", str(t), "--output", str(out), "--blocks", "2", "--cells", "2"]) == 0
    assert main(["sample", str(out), "-n", "4", "-o", str(tmp_path / "p.pdt"), "--duration", "0.2"]) == 0
    from featurenet_amd.fm.products import ProductSet

    assert ProductSet(tmp_path / "p.pdt").nbProducts == 4


@need_rt
def test_run_end_to_end_tiny(tmp_path, capsys):
    cfg = tmp_path / "c.json"
    cfg.write_text(json.dumps({"attacks": [], "synthetic_sizes": [128, 32], "devices": "cpu"}))
    rc = main(["run", "--config", str(cfg), "-n", "1x1x3", "-t", "1", "-b", str(tmp_path / "prod"), "-i", "0.2",
               "-e", "1", "-s", "0.5"])
    assert rc == 0
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert res["generations"] == 1
    assert os.path.isdir(res["session"])
