"""Measured collective tuning (parallel/comm_tuning.py): bench/comm_bench.py --write-tuning
stores the bucket size and P2P crossover per world size; bench.py --bucket-mb auto and the
P2P path read them back, and fall back to their defaults when the world size was never
measured (the P2P path is never switched on by a 1-rank measurement)."""
import json

from cloudtik_amd.parallel import comm_tuning as CT


def test_record_and_read_back(tmp_path, monkeypatch):
    p = str(tmp_path / "tuning.json")
    monkeypatch.setenv("CLOUDTIK_COMM_TUNING", p)
    assert CT.bucket_mb(8, 64.0) == 64.0 and CT.p2p_bytes(8) == 0
    CT.record(8, 48 * CT.MiB, 1 << 20, rccl="2.26.6")
    CT.record(1, 1 * CT.MiB, 4 << 20)
    d = json.load(open(p))
    assert set(d) == {"1", "8"} and d["8"]["rccl"] == "2.26.6"
    assert CT.bucket_mb(8, 64.0) == 48.0 and CT.p2p_bytes(8) == 1 << 20
    assert CT.bucket_mb(1, 64.0) == 4.0            # clamped to the 4 MiB floor
    assert CT.p2p_bytes(1) == 0                    # a 1-rank crossover never enables P2P
    assert CT.bucket_mb(4, 8.0) == 8.0             # never measured: the default


def test_bench_resolves_auto_buckets(tmp_path, monkeypatch):
    import bench
    monkeypatch.setenv("CLOUDTIK_COMM_TUNING", str(tmp_path / "t.json"))
    assert bench.resolve_bucket_mb("auto", 8, 64.0) == 64.0
    assert bench.resolve_bucket_mb("16", 8, 64.0) == 16.0
    CT.record(8, 32 * CT.MiB, None)
    assert bench.resolve_bucket_mb("auto", 8, 64.0) == 32.0
    assert bench.parse(["--bucket-mb", "auto"]).bucket_mb == "auto"
