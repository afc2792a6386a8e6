"""Single-node cluster front end (deploy/node.yaml -> launch commands)."""
import os
import sys

from pyspark_tf_gke_amd.runtime import node

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_node_yaml_roles():
    cfg = node.load(os.path.join(ROOT, "deploy", "node.yaml"))
    assert cfg["node"]["gpus"] == 8 and cfg["spark"]["executors"] == 8 and cfg["tensorflow"]["workers"] == 8
    cmd, env, ranks = node.commands(cfg, "spark", ["app.py"])
    assert ranks == 1 and "--num-executors" in cmd and cmd[cmd.index("--num-executors") + 1] == "8"
    assert "spark.driver.port=7078" in cmd and cmd[-1] == "app.py"
    cmd, env, ranks = node.commands(cfg, "train", ["--epochs", "1"])
    assert ranks == 8 and cmd[0] == sys.executable and cmd[1].endswith("train_tf_ps.py")
    assert cmd[cmd.index("--strategy") + 1] == "mirrored" and env["MASTER_PORT"] == "29500"
    cmd, env, ranks = node.commands(cfg, "joint", [])
    assert ranks == 8 and cmd[1].endswith("etl_to_train.py")


def test_node_rejects_oversubscription(tmp_path):
    p = tmp_path / "n.yaml"
    p.write_text("node: {gpus: 2}\nspark: {executors: 4}\n")
    try:
        node.load(str(p))
    except ValueError:
        return
    raise AssertionError("expected ValueError")
