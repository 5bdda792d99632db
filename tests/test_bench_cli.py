"""bench.py's rank handling on CPU (no GPU call is made on these paths).

* WORLD_SIZE set by a launcher and a different --gpus: exit non-zero with a message,
  never a line that labels an N-rank run as M GPUs.
* --gpus N > 1 without a launcher: bench.py starts N ranks under torch.distributed.run
  itself.  Here (no HIP device) every rank then stops at the device check, which proves
  the ranks were started and reached the device mapping.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    env.update(kw)
    return env


def test_world_size_mismatch_refused():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--steps", "1"],
                         capture_output=True, text=True, timeout=300,
                         env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert out.returncode != 0
    assert "--gpus 1 but the launcher started WORLD_SIZE=2" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_gpus_n_starts_n_ranks():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--no-cpu",
                          "--e2e", "0"], capture_output=True, text=True, timeout=300,
                         env=_env(CUDA_VISIBLE_DEVICES=""))
    assert out.returncode != 0                    # no device here: both ranks fail loudly
    # torch.distributed.run reports each failed local rank; both reached the device check
    assert out.stderr.count("needs a HIP device") >= 1
    assert "local_rank: 0" in out.stderr and "local_rank: 1" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]
