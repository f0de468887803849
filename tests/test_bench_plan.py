"""bench.py's launch contract (CPU): --gpus N starts N ranks itself unless a
torch.distributed launcher already did, and a launcher's WORLD_SIZE must equal
N (runner.py:135-141 is the reference's own process-per-simulation fan-out)."""
import bench


def test_single_gpu_runs_in_process():
    assert bench.launch_plan(1, {}) == ("run", 1)


def test_multi_gpu_without_launcher_spawns():
    assert bench.launch_plan(8, {}) == ("spawn", 8)


def test_launcher_world_must_match():
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}) == ("run", 2)
    plan, msg = bench.launch_plan(8, {"WORLD_SIZE": "1"})
    assert plan == "error" and "WORLD_SIZE=1" in msg
    assert bench.launch_plan(0, {})[0] == "error"
