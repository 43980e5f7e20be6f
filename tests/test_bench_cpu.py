"""bench.py's CPU baseline leg, on small samples (no GPU): the record the N = 1
and N > 1 JSON lines carry (one storage per server thread, and 8
server threads with 8 storages beside the multi-GPU figure)."""
import bench


def test_cpu_baseline_one_thread_record(oracle_mod):
    rec = bench.cpu_baseline([0, 5000, 20000, 5000], 2000, 4, [3000, 4000])
    assert rec["cores"] == 1 and rec["kind"] == "port" and rec["value"] > 0
    assert rec["eight_threads"]["cores"] == 8 and rec["eight_threads"]["value"] > 0
    assert [s["n"] for s in rec["vector_storage"]["samples"]] == [3000, 4000]
    assert "measured_1e6" not in rec["vector_storage"]  # only this run's samples


def test_cpu_baseline_eight_servers_record(oracle_mod):
    rec = bench.cpu_baseline([0, 5000, 20000, 5000], 2000, 4, [], servers=8)
    assert rec["cores"] == 8 and rec["kind"] == "port" and rec["value"] > 0
    assert rec["one_thread"]["cores"] == 1 and rec["one_thread"]["value"] > 0
    assert "vector_storage" not in rec and "host_cpu" in rec
