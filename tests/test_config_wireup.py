"""T1: CLI parity and scheduler wire-up parsing with fake environments (survey §4, App. D, Q1/Q2/Q5)."""
import pytest

from pytorch_ddp_mnist_amd import config as C
from pytorch_ddp_mnist_amd.parallel import wireup as W


def test_mp_defaults_match_reference():
    cfg = C.configure([])
    nested = cfg.to_nested()
    assert nested["trainer"] == {"batch_size": 128, "wireup_method": "nccl-slurm", "parallel": False,
                                 "device": 0, "n_epochs": 1, "num_workers": 0}
    assert nested["data"]["limit"] is None
    assert nested["data"]["label_map"] == [0, 1, 0, 0, 2, 3, 1, 4]
    assert "path" not in nested["data"]


def test_mp_flags_override_only_when_given():
    cfg = C.configure(["--wireup_method", "gloo", "--batch_size", "64", "--n_epochs", "3", "--num_workers", "2",
                       "--data_path", "/x", "--data_limit", "100", "--parallel", "--hdf5"])
    assert (cfg.wireup_method, cfg.batch_size, cfg.n_epochs, cfg.num_workers) == ("gloo", 64, 3, 2)
    assert cfg.data_path == "/x" and cfg.data_limit == 100 and cfg.parallel and cfg.hdf5
    assert cfg.to_nested()["data"]["path"] == "/x"


def test_mpich_only_in_pnetcdf_cli():
    with pytest.raises(SystemExit):
        C.configure(["--wireup_method", "mpich"])
    assert C.configure(["--wireup_method", "mpich"], pnetcdf=True).wireup_method == "mpich"


@pytest.mark.parametrize("argv", [["--local_rank", "3"], ["--local-rank=3"], ["--local-rank", "3"]])
def test_gpu_tutorial_local_rank_spellings(argv):
    cfg = C.configure_gpu_tutorial(argv)
    assert cfg.local_rank == 3 and cfg.batch_size == 128 and cfg.n_epochs == 10


def test_gpu_tutorial_local_rank_env(monkeypatch):
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert C.configure_gpu_tutorial([]).local_rank == 5


def test_additive_flags():
    cfg = C.configure(["--model", "lenet5", "--dtype", "bf16", "--momentum", "0.9", "--no_graph", "--no_save",
                       "--bucket_cap_kb", "64", "--synthetic"])
    assert cfg.model == "lenet5" and cfg.dtype == "bf16" and cfg.momentum == 0.9
    assert not cfg.graph and cfg.save_path is None and cfg.bucket_cap_kb == 64 and cfg.data_format == "synthetic"


def test_allreduce_and_overlap_plan_flags():
    from pytorch_ddp_mnist_amd.engine.native import resolve_plan
    cfg = C.configure(["--allreduce", "oneshot", "--plan", "overlap"])
    assert cfg.allreduce == "oneshot" and cfg.plan == "overlap" and resolve_plan(cfg.plan) == "overlap"
    assert C.configure([]).allreduce == "rccl"
    with pytest.raises(SystemExit):
        C.configure(["--allreduce", "nccl"])


# ------------------------------------------------------------------------------------ wire-up
def test_slurm_full_env():
    env = {"SLURM_LAUNCH_NODE_IPADDR": "10.0.0.7", "SLURM_SRUN_COMM_PORT": "4242", "SLURM_NTASKS": "8",
           "SLURM_PROCID": "5", "SLURM_LOCALID": "1"}
    w = W.resolve("nccl-slurm", env)
    assert (w.master_addr, w.master_port, w.world_size, w.rank, w.local_rank) == ("10.0.0.7", 4242, 8, 5, 1)


def test_slurm_tasks_per_node_is_parsed_not_string_multiplied():  # quirk Q2
    env = {"SLURM_LAUNCH_NODE_IPADDR": "h", "SLURM_JOB_NUM_NODES": "2", "SLURM_TASKS_PER_NODE": "4(x2)",
           "SLURM_PROCID": "0"}
    assert W.resolve("nccl-slurm", env).world_size == 8
    env["SLURM_TASKS_PER_NODE"] = "4(x2),3"
    assert W.resolve("nccl-slurm", dict(env, SLURM_JOB_NUM_NODES="3")).world_size == 11
    env2 = {"SLURM_LAUNCH_NODE_IPADDR": "h", "SLURM_JOB_NUM_NODES": "3", "SLURM_NTASKS_PER_NODE": "4",
            "SLURM_PROCID": "2"}
    assert W.resolve("nccl-slurm", env2).world_size == 12
    assert W.parse_slurm_tasks_per_node("2(x3),1") == [2, 2, 2, 1]


def test_slurm_missing_env_errors():
    with pytest.raises(W.WireupError):
        W.resolve("nccl-slurm", {})
    with pytest.raises(W.WireupError):
        W.resolve("nccl-slurm", {"SLURM_LAUNCH_NODE_IPADDR": "h"})


def test_openmpi_pmix_uri_is_subscripted():  # quirk Q1
    env = {"PMIX_SERVER_URI2": "pmix-server.77;tcp4://192.168.1.9:5555", "OMPI_COMM_WORLD_SIZE": "4",
           "OMPI_COMM_WORLD_RANK": "2", "OMPI_COMM_WORLD_LOCAL_RANK": "2"}
    w = W.resolve("nccl-openmpi", env)
    assert (w.master_addr, w.master_port, w.world_size, w.rank, w.local_rank) == ("192.168.1.9", 29500, 4, 2, 2)
    with pytest.raises(W.WireupError):
        W.resolve("nccl-openmpi", {"OMPI_COMM_WORLD_SIZE": "4", "OMPI_COMM_WORLD_RANK": "0"})


@pytest.mark.parametrize("method", ["nccl-mpich", "mpich"])
def test_mpich_pmi(method):
    w = W.resolve(method, {"PMI_SIZE": "4", "PMI_RANK": "3"})
    assert (w.master_addr, w.master_port, w.world_size, w.rank) == ("localhost", 29500, 4, 3)
    w1 = W.resolve(method, {})
    assert (w1.world_size, w1.rank) == (1, 0)


def test_gloo_precedence():
    env = {"OMPI_COMM_WORLD_SIZE": "2", "OMPI_COMM_WORLD_RANK": "1", "PMI_SIZE": "9", "PMI_RANK": "8",
           "PMIX_SERVER_URI2": "x;tcp4://1.2.3.4:77"}
    w = W.resolve("gloo", env)
    assert (w.master_addr, w.world_size, w.rank) == ("1.2.3.4", 2, 1)
    assert W.resolve("gloo", {"WORLD_SIZE": "3", "RANK": "2", "MASTER_ADDR": "m", "MASTER_PORT": "1"}).master_port == 1


def test_bad_rank_and_method():
    with pytest.raises(W.WireupError):
        W.resolve("gloo", {"WORLD_SIZE": "2", "RANK": "2"})
    with pytest.raises(NotImplementedError):
        W.resolve("nccl-foo", {})


def test_export_and_local_rank():
    env = {}
    w = W.apply("nccl-mpich", dict(PMI_SIZE="2", PMI_RANK="1"))
    w.export(env)
    assert env["WORLD_SIZE"] == "2" and env["RANK"] == "1" and env["MASTER_ADDR"] == "localhost"
    assert W.pick_local_rank(w, 8) == 1
    assert W.pick_local_rank(W.resolve("gloo", {"WORLD_SIZE": "16", "RANK": "13"}), 8) == 5
