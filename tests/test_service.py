"""REST task service: reference routes, SQLite store, worker pipeline (CPU, tiny)."""
import os

import pytest

REF = "/root/reference"


def test_store_concurrent_field_updates(tmp_path):
    from featurenet_amd.service.store import TaskStore

    s = TaskStore(tmp_path / "t.db")
    t = s.create({"task_name": "a b", "dataset": "mnist"})
    assert t["task_name"] == "a_b" and t["status"] == "init"
    s.update(t["task_id"], fm="x.xml")
    s2 = TaskStore(tmp_path / "t.db")          # a second "process" view
    s2.update(t["task_id"], "fm_complete", pdt="y.pdt")
    got = s.get(t["task_id"])
    assert got["fm"] == "x.xml" and got["pdt"] == "y.pdt" and got["status"] == "fm_complete"
    assert len(s.all()) == 1 and s.delete_all() == 1 and s.all() == []


@pytest.mark.skipif(not os.path.isfile(f"{REF}/ui/back/samples.db"), reason="no reference samples.db")
def test_store_opens_reference_db(tmp_path):
    import shutil

    from featurenet_amd.service.store import TaskStore

    dst = tmp_path / "samples.db"
    shutil.copy(f"{REF}/ui/back/samples.db", dst)      # plain SQLite, read as data
    assert isinstance(TaskStore(dst).all(), list)


def test_generated_template_matches_reference():
    from featurenet_amd.fm.space import SearchSpace

    if not os.path.isfile(f"{REF}/main_1block_nas.xml"):
        pytest.skip("no reference template")
    assert SearchSpace().xml() == open(f"{REF}/main_1block_nas.xml").read()


def test_rest_routes_and_worker_pipeline(tmp_path):
    from fastapi.testclient import TestClient

    from featurenet_amd import _native
    from featurenet_amd.service.server import create_app
    from featurenet_amd.service.worker import run_task

    if not _native.runtime_available():
        pytest.skip("native runtime not built")
    db, base = str(tmp_path / "s.db"), str(tmp_path / "products")
    app = create_app(db, base, spawn_workers=False)
    c = TestClient(app)
    r = c.post("/sample/", json={"data": {"task_name": "t1", "dataset": "mnist", "max_sampling_time": 0.3,
                                          "nb_initial_config": 3, "max_nb_cells": 1, "max_nb_blocks": 1,
                                          "nb_training_iterations": 1, "synthetic_sizes": [128, 32]}})
    tid = r.json()["task_id"]
    assert c.get("/sample/").json()[0]["task_id"] == tid
    done = run_task(app.state.store, tid, base, devices=["cpu"])
    assert done["status"] == "generation_complete", done.get("error")
    full = c.get(f"/sample/{tid}", params={"full": 1}).json()
    assert len(full["models"]) == 3
    assert c.get("/sample/").json()[0]["nb_valid_elements"] >= 1
    name = full["models"][0]["name"]
    g = c.get(f"/sample/{tid}/product/{name}/graph")
    assert g.status_code == 200 and g.text.startswith("<svg")
    m = c.get(f"/sample/{tid}/product/{name}/model")
    assert m.status_code == 200 and len(m.content) > 100
    assert "<html>" in c.get("/").text
    assert c.delete("/sample/").json() == 1


def test_store_rejects_path_escape_and_server_keys(tmp_path):
    """client task names are one safe path component; server-owned fields are dropped."""
    from featurenet_amd.service.store import TaskStore, safe_name

    assert safe_name("../../etc x") == "etc_x"
    s = TaskStore(tmp_path / "t.db")
    t = s.create({"task_name": "../../evil", "products": "/etc", "fm_template": "/etc/passwd", "pdt": "/x",
                  "dataset": "mnist"})
    assert t["task_name"] == "evil"
    for k in ("products", "fm_template", "pdt"):
        assert k not in s.get(t["task_id"])


def test_worker_cap_and_bad_product_id(tmp_path):
    from fastapi.testclient import TestClient

    from featurenet_amd.service.server import create_app

    app = create_app(str(tmp_path / "s.db"), str(tmp_path / "p"), spawn_workers=False)
    c = TestClient(app)
    tid = c.post("/sample/", json={"data": {"task_name": "t"}}).json()["task_id"]
    assert c.get(f"/sample/{tid}/product/..%2F..%2Fx/model").status_code in (400, 404)
    assert c.get(f"/sample/{tid}/product/a..b/model").status_code == 400

    class Running:
        def poll(self):
            return None

        def terminate(self):
            self.t = True

        def wait(self, timeout=None):
            return 0

    app2 = create_app(str(tmp_path / "s2.db"), str(tmp_path / "p2"), spawn_workers=True, max_workers=1)
    app2.state.workers["x"] = w = Running()
    c2 = TestClient(app2)
    assert c2.post("/sample/", json={"data": {"task_name": "t"}}).status_code == 429
    c2.delete("/sample/")                                   # DELETE stops running workers
    assert getattr(w, "t", False) and app2.state.workers == {}


def test_server_binds_localhost_by_default():
    import inspect

    from featurenet_amd.service.server import serve

    assert inspect.signature(serve).parameters["host"].default == "127.0.0.1"


def _catalogue_keys(node, out):
    out.append(node)
    for c in node.get("children", []):
        _catalogue_keys(c, out)
    return out


def test_fm_builder_routes_produce_a_sampleable_feature_model(tmp_path):
    """FM builder (reference ui/src/pages/fm.js + util.js buildTree): the checked cell
    features become a SPLOT model that parses, extends to B x C and samples."""
    from fastapi.testclient import TestClient

    from featurenet_amd import _native
    from featurenet_amd.fm import extend, splot
    from featurenet_amd.service.server import create_app

    app = create_app(str(tmp_path / "s.db"), str(tmp_path / "p"), spawn_workers=False)
    c = TestClient(app)
    cat = c.get("/fm/catalogue").json()
    nodes = _catalogue_keys(cat[0], [])
    keys = [n["key"] for n in nodes]
    assert len(keys) == len(set(keys))                                   # unique keys (reference reuses some)
    assert any(n["title"] == "Convolution" for n in nodes) and any(n["disabled"] for n in nodes)
    sel = [n["key"] for n in nodes if not n["disabled"] and not any(
        s in n["key"] for s in ("dense", "pooling", "recurrence", "flatten", "padding/fillsize"))]
    r = c.post("/fm/build", json={"checked": sel})
    assert r.status_code == 200 and r.headers["content-disposition"].endswith('fm.xml"')
    fm = splot.loads(r.text)
    names = set(fm.names())
    assert "Block[k]_Element[i]_Cell_Input1_Convolution_kernel_3x3" in names
    assert not any("Dense" in n for n in names)
    assert "C7:~Architecture  or  ~Block[k]_Element[i]_Cell_Input1_Zeros" in r.text
    src = tmp_path / "fm.xml"
    src.write_text(r.text)
    extend.generate_featuretree(src, tmp_path / "fm_2_2.xml", 2, 2)
    big = splot.load(tmp_path / "fm_2_2.xml")
    assert "Block2_Element2_Cell_Input2_Identity" in set(big.names())
    if _native.runtime_available():
        from featurenet_amd.fm.sampler import sample_products

        res = sample_products(big, 4, duration_s=0.5, seed=0)
        prods = res["products"]
        assert len(prods) >= 1
        for prod in prods:
            chosen = {res["labels"][abs(v) - 1] for v in prod if v > 0}
            assert big.is_valid(chosen)
    # unchecking Zeros drops the constraint that names it
    r2 = c.post("/fm/build", json={"checked": [k for k in sel if "zeros" not in k]})
    assert "Input1_Zeros" not in r2.text
    assert c.post("/fm/build", json={"checked": "cell"}).status_code == 400
