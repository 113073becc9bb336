"""Deployment generators (reference docker/local.sh, docker/client/script/submit.py)."""
import yaml

from parameter_server_amd import deploy


def test_docker_local_node_specs():
    cmds = deploy.docker_local(2, 3, "/a.conf", "/d", "/m", ["-num_threads", "4"])
    assert len(cmds) == 6
    roles = [c[c.index("-my_node") + 1].split(",")[0] for c in cmds]
    assert roles == ["role:SCHEDULER"] + ["role:SERVER"] * 2 + ["role:WORKER"] * 3
    ids = [c[c.index("-my_node") + 1].split("id:")[1] for c in cmds]
    assert ids == ["'H'", "'S0'", "'S1'", "'W0'", "'W1'", "'W2'"]
    assert all("-num_threads" in c and c[c.index("-scheduler") + 1] == c[c.index("-my_node") + 1]
               for c in cmds[:1])


def test_k8s_gpu_manifest():
    objs = yaml.safe_load_all(deploy._yaml(deploy.k8s_gpu(4, ["bench.py", "--gpus", "8"])))
    svc, job = list(objs)
    assert svc["kind"] == "Service" and svc["spec"]["clusterIP"] == "None"
    spec = job["spec"]
    assert spec["completions"] == 4 and spec["completionMode"] == "Indexed"
    c = spec["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    cmd = c["command"][-1]
    assert "--nnodes=4" in cmd and "--nproc-per-node=8" in cmd and "bench.py" in cmd
    assert "$(JOB_COMPLETION_INDEX)" in cmd


def test_k8s_runtime_roles(tmp_path):
    objs = deploy.k8s_runtime(2, 5, "linear_method { }")
    kinds = [o["kind"] for o in objs]
    assert kinds == ["ConfigMap", "Service", "Pod", "StatefulSet", "StatefulSet"]
    assert objs[3]["spec"]["replicas"] == 2 and objs[4]["spec"]["replicas"] == 5
    yaml.safe_load_all(deploy._yaml(objs))


def test_cli_prints(capsys):
    assert deploy.main(["dockerfile"]) == 0
    assert "gfx950" in capsys.readouterr().out
    assert deploy.main(["docker-local", "1", "1", "a.conf", "d", "m"]) == 0
    out = capsys.readouterr().out
    assert out.count("docker run") == 3
