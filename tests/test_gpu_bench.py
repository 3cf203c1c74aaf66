"""bench.py end to end on the GPU at small sizes: every resident mode through
both engines (one process per GPU, and the multi-device context the Go shim
uses), strong scaling by --total-gib, and host ingest through the capped,
NUMA-bound pinned pool.  Each run checks its own blocks against the oracle and
exits non-zero on a difference (bench.py check_resident / full_check), so a
zero exit and a well-formed line are the assertions here."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                          "--no-cpu"] + list(args), env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("engine", ["process", "mctx"])
@pytest.mark.parametrize("mode", ["seal", "open", "decrypt", "crc"])
def test_resident_modes(engine, mode):
    rec = bench("--engine", engine, "--mode", mode, "--blocks", "48", "--verify", "3")
    assert rec["value"] > 0 and rec["n_gpus"] >= 1 and rec["scaling"] == "weak"
    assert rec["full_check"]["blocks"] == 48 * rec["n_gpus"]
    assert rec["roofline"]["frac"] > 0 and rec["roofline"]["kernel_launches"] >= 2
    if mode != "seal":
        assert "setup" in rec["full_check"]["what"]
    if mode in ("open", "decrypt"):
        assert "ETAG" in rec["full_check"]["what"] and rec["full_check"]["plaintext_samples"] >= 3


def test_strong_scaling_loops_over_the_resident_batch():
    rec = bench("--engine", "mctx", "--mode", "open", "--total-gib", str(100 * 4 / 1024), "--blocks", "32")
    assert rec["scaling"] == "strong" and rec["config"]["resident_blocks_per_gpu"] == 32
    assert rec["config"]["blocks_per_gpu"] * rec["n_gpus"] >= 100
    assert rec["roofline"]["kernel_launches"] >= 2 * 4  # 2 steps x 4 loops (100 blocks / 32 resident)


@pytest.mark.parametrize("engine", ["process", "mctx"])
def test_host_ingest_through_the_capped_pool(engine):
    rec = bench("--engine", engine, "--mem", "host", "--blocks", "40", "--host-pool-gib", str(16 * 4 / 1024),
                "--verify", "2")
    cfg = rec["config"]
    assert cfg["pool_blocks_per_gpu"] == 16 and cfg["blocks_per_gpu"] == 40
    assert cfg["pinned_bytes_per_process"] <= rec["n_gpus"] * (2 * 16 * (4 << 20) + 16 * 512)
    assert rec["full_check"]["blocks"] == 16 * rec["n_gpus"]
    assert 0 < rec["roofline"]["frac_of_link"] < 1.0
    assert all(n["pool_node"] != -2 for n in cfg["numa"])
