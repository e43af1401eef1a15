"""World-2 run of the product's multi-GPU code on the GPU box (one card, two
ranks on cuda:0, gloo): ShardedIndexFlat / ShardedIndexIVFFlat equal one index
over the whole corpus, and FusedTrainStep's data-parallel gradient hook
produces the rank-mean gradient with replicas staying identical (gloo carries
host copies of the device buffers).  The RCCL branches of dist.py
(all_gather_into_tensor / all_reduce / all_to_all on device buffers, and the
all_reduce captured inside the DIN step's HIP graph) run here too, at world 1
over the "nccl" backend (test_rccl_branch_world1, tests/rccl_world1_worker.py).
What no test here covers is RCCL across several GPUs (the driver's 8-GPU
scaling run).  The ranks run as child processes of torch.distributed.run."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_world2_sharded_search_and_dp_hook(gpu, tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_gpu_worker.py"), str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(2)]
    for x in res:
        assert x["world"] == 2
        for m in (0, 1):
            assert x[f"flat{m}_I_equal"] and x[f"flat{m}_D_equal"], (m, x)
            assert x[f"flat{m}_own_equal"], (m, x)
        assert x["ivf_centroids_equal"] and x["ivf_I_equal"] and x["ivf_D_equal"], x
        assert x["dp_grad_rel_err"] < 1e-6, x
        assert x["dp_replica_param_diff"] == 0.0, x
    assert res[0]["flat0_local_rows"] + res[1]["flat0_local_rows"] == 50_001


def test_rccl_branch_world1(gpu, tmp_path):
    """The RCCL (`nccl` backend) branches of newsrecommend_amd.dist on device
    buffers, at world 1 on the one-GPU box (RCCL refuses two ranks on one
    card): all_gather_results, scatter_results and all_reduce_mean_ equal the
    gloo branches bit for bit, and the gradient all_reduce captured inside the
    FusedTrainStep graph leaves the steps bit-identical to un-hooked ones."""
    out = tmp_path / "rccl.json"
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_world1_worker.py"), str(out)], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    x = json.load(open(out))
    assert x["backend"] == "nccl" and x["gloo_backend"] == "gloo", x
    for key in ("all_gather_device", "all_gather_equal", "scatter_equal", "merge_equal", "all_reduce_equal",
                "dp_graph_equal", "dp_graph_loss_equal"):
        assert x[key], (key, x)
