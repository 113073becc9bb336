"""Container / cluster deployment generators.

Reference: docker/local.sh (one container per node on the docker0 bridge:
scheduler H, servers S*, workers W*, ``-my_node`` / ``-scheduler`` node specs)
and docker/client/script/submit.py (Kubernetes v1beta1 pods + replication
controllers for ``submit S W batch|online data out``).

Two deployment shapes here:

* ``docker-local S W app.conf data_dir model_dir [args]`` — the reference's
  container-per-node runtime (CPU control plane / plumbing runs): prints, or with
  ``--run`` executes, one ``docker run`` per node.
* ``k8s-gpu --nodes N`` — the MI355X-native shape: one pod per 8-GPU node
  (``amd.com/gpu: 8``, ``/dev/kfd`` + ``/dev/dri``), an Indexed Job so pod i is
  node rank i, a headless Service for the rendezvous, and ``torchrun
  --nproc-per-node 8`` inside the pod (one process per GPU, RCCL over xGMI inside
  the node, RCCL over the NICs across nodes).
* ``k8s-runtime S W`` — the reference's role layout (scheduler / servers /
  workers as separate pods) for the CPU runtime, with modern apps/v1 objects.

All generators print YAML / shell to stdout; nothing talks to a cluster.
"""
from __future__ import annotations

import argparse
import shlex
import sys

IMAGE = "parameter-server-amd:rocm7"


# ----------------------------------------------------------------- docker (local)
def docker_local(num_servers: int, num_workers: int, app: str, data: str, model: str,
                 extra: list[str], *, ip: str = "172.17.0.1", port: int = 8000,
                 image: str = IMAGE) -> list[list[str]]:
    """One ``docker run`` argv per node (scheduler first), reference docker/local.sh."""
    sch = f"role:SCHEDULER,hostname:'{ip}',port:{port},id:'H'"
    mounts = ["-v", f"{app}:/app.conf", "-v", f"{data}:/data", "-v", f"{model}:/model"]
    args = ["-app_file", "/app.conf", "-num_servers", str(num_servers), "-num_workers",
            str(num_workers)] + list(extra)
    cmds = []
    for i in range(num_servers + num_workers + 1):
        p = port + i
        if i == 0:
            node = sch
        elif i <= num_servers:
            node = f"role:SERVER,hostname:'{ip}',port:{p},id:'S{i - 1}'"
        else:
            node = f"role:WORKER,hostname:'{ip}',port:{p},id:'W{i - 1 - num_servers}'"
        cmds.append(["docker", "run", "--rm", "-p", f"{p}:{p}", "--name", f"psamd-n{i}", *mounts,
                     image, "python", "-m", "parameter_server_amd.app.main", "-my_node", node,
                     "-scheduler", sch, "-bind_to", str(p), *args])
    return cmds


# ------------------------------------------------------------------- kubernetes
def _yaml(objs: list[dict]) -> str:
    import yaml

    return "---\n".join(yaml.safe_dump(o, sort_keys=False) for o in objs)


def k8s_gpu(nodes: int, command: list[str], *, name: str = "psamd", image: str = IMAGE,
            gpus_per_node: int = 8, port: int = 29500, namespace: str = "default") -> list[dict]:
    """Headless Service + Indexed Job: pod i = node rank i, torchrun with one
    process per GPU inside each pod."""
    svc = {"apiVersion": "v1", "kind": "Service",
           "metadata": {"name": name, "namespace": namespace},
           "spec": {"clusterIP": "None", "selector": {"app": name},
                    "ports": [{"name": "rdzv", "port": port}]}}
    master = f"{name}-0.{name}.{namespace}.svc"
    run = ["python", "-m", "torch.distributed.run", f"--nnodes={nodes}",
           f"--nproc-per-node={gpus_per_node}", "--node-rank=$(JOB_COMPLETION_INDEX)",
           f"--master-addr={master}", f"--master-port={port}"] + list(command)
    container = {
        "name": "trainer", "image": image,
        "command": ["bash", "-c", " ".join(shlex.quote(c) if "$(" not in c else c for c in run)],
        "env": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"},
                {"name": "NCCL_SOCKET_IFNAME", "value": "eth0"}],
        "resources": {"limits": {"amd.com/gpu": gpus_per_node},
                      "requests": {"amd.com/gpu": gpus_per_node}},
        "ports": [{"containerPort": port}],
        "securityContext": {"capabilities": {"add": ["SYS_PTRACE"]}},
        "volumeMounts": [{"name": "kfd", "mountPath": "/dev/kfd"},
                         {"name": "dri", "mountPath": "/dev/dri"},
                         {"name": "shm", "mountPath": "/dev/shm"}],
    }
    job = {"apiVersion": "batch/v1", "kind": "Job",
           "metadata": {"name": name, "namespace": namespace},
           "spec": {"completions": nodes, "parallelism": nodes, "completionMode": "Indexed",
                    "backoffLimit": 0,
                    "template": {"metadata": {"labels": {"app": name}},
                                 "spec": {"subdomain": name, "restartPolicy": "Never",
                                          "hostIPC": True, "containers": [container],
                                          "volumes": [
                                              {"name": "kfd", "hostPath": {"path": "/dev/kfd"}},
                                              {"name": "dri", "hostPath": {"path": "/dev/dri"}},
                                              {"name": "shm", "emptyDir": {"medium": "Memory"}}]}}}}
    return [svc, job]


def k8s_runtime(num_servers: int, num_workers: int, app_conf: str, *, name: str = "psamd-rt",
                image: str = IMAGE, port: int = 8000, namespace: str = "default") -> list[dict]:
    """Reference submit.py role layout: a scheduler Pod + Service, and server /
    worker StatefulSets whose pods address the scheduler by its service name."""
    sch_host = f"{name}-scheduler.{namespace}.svc"
    sch = f"role:SCHEDULER,hostname:'{sch_host}',port:{port},id:'H'"
    common = ["-app_file", "/config/app.conf", "-num_servers", str(num_servers),
              "-num_workers", str(num_workers), "-scheduler", sch]
    cfg_vol = {"name": "config", "configMap": {"name": f"{name}-config"}}
    cm = {"apiVersion": "v1", "kind": "ConfigMap",
          "metadata": {"name": f"{name}-config", "namespace": namespace},
          "data": {"app.conf": app_conf}}
    svc = {"apiVersion": "v1", "kind": "Service",
           "metadata": {"name": f"{name}-scheduler", "namespace": namespace},
           "spec": {"selector": {"app": name, "role": "scheduler"},
                    "ports": [{"port": port}]}}

    def pod_spec(role, node_expr):
        cmd = ("python -m parameter_server_amd.app.main -my_node \"" + node_expr + "\" " +
               " ".join(shlex.quote(c) for c in common))
        return {"containers": [{"name": role, "image": image, "command": ["bash", "-c", cmd],
                                "ports": [{"containerPort": port}],
                                "volumeMounts": [{"name": "config", "mountPath": "/config"}]}],
                "volumes": [cfg_vol]}

    sched = {"apiVersion": "v1", "kind": "Pod",
             "metadata": {"name": f"{name}-scheduler", "namespace": namespace,
                          "labels": {"app": name, "role": "scheduler"}},
             "spec": {**pod_spec("scheduler", sch), "restartPolicy": "Never"}}
    objs = [cm, svc, sched]
    for role, n, prefix in (("server", num_servers, "S"), ("worker", num_workers, "W")):
        node = (f"role:{role.upper()},hostname:'$(hostname -i)',port:{port},"
                f"id:'{prefix}'$(hostname | sed 's/.*-//')")
        objs.append({"apiVersion": "apps/v1", "kind": "StatefulSet",
                     "metadata": {"name": f"{name}-{role}", "namespace": namespace},
                     "spec": {"replicas": n, "serviceName": f"{name}-{role}",
                              "selector": {"matchLabels": {"app": name, "role": role}},
                              "template": {"metadata": {"labels": {"app": name, "role": role}},
                                           "spec": pod_spec(role, node)}}})
    return objs


DOCKERFILE = """\
# MI355X (gfx950) image: ROCm PyTorch base + this package built in-tree.
FROM rocm/pytorch:latest
ENV PYTORCH_ROCM_ARCH=gfx950 HSA_ENABLE_IPC_MODE_LEGACY=0
WORKDIR /opt/psamd
COPY . /opt/psamd
RUN python -m parameter_server_amd._build
ENV PYTHONPATH=/opt/psamd
"""


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m parameter_server_amd.deploy")
    sub = ap.add_subparsers(dest="cmd", required=True)
    d = sub.add_parser("docker-local")
    d.add_argument("num_servers", type=int)
    d.add_argument("num_workers", type=int)
    d.add_argument("app")
    d.add_argument("data")
    d.add_argument("model")
    d.add_argument("extra", nargs=argparse.REMAINDER)
    d.add_argument("--ip", default="172.17.0.1")
    d.add_argument("--image", default=IMAGE)
    d.add_argument("--run", action="store_true", help="execute instead of printing")
    g = sub.add_parser("k8s-gpu")
    g.add_argument("--nodes", type=int, required=True)
    g.add_argument("--gpus-per-node", type=int, default=8)
    g.add_argument("--image", default=IMAGE)
    g.add_argument("--name", default="psamd")
    g.add_argument("command", nargs=argparse.REMAINDER)
    r = sub.add_parser("k8s-runtime")
    r.add_argument("num_servers", type=int)
    r.add_argument("num_workers", type=int)
    r.add_argument("app_conf", help="path of the text-format app config to ship")
    r.add_argument("--image", default=IMAGE)
    sub.add_parser("dockerfile")
    a = ap.parse_args(argv)
    if a.cmd == "docker-local":
        cmds = docker_local(a.num_servers, a.num_workers, a.app, a.data, a.model, a.extra,
                            ip=a.ip, image=a.image)
        if not a.run:
            print("\n".join(" ".join(shlex.quote(c) for c in cmd) + " &" for cmd in cmds))
            print("wait")
            return 0
        import subprocess

        procs = [subprocess.Popen(c) for c in cmds]
        return max(p.wait() for p in procs)
    if a.cmd == "k8s-gpu":
        cmd = a.command[1:] if a.command[:1] == ["--"] else a.command
        print(_yaml(k8s_gpu(a.nodes, cmd or ["bench.py", "--gpus", str(a.gpus_per_node)],
                            name=a.name, image=a.image, gpus_per_node=a.gpus_per_node)))
        return 0
    if a.cmd == "k8s-runtime":
        with open(a.app_conf) as f:
            conf = f.read()
        print(_yaml(k8s_runtime(a.num_servers, a.num_workers, conf, image=a.image)))
        return 0
    sys.stdout.write(DOCKERFILE)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
