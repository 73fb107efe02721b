"""The one collective of the path on real hardware: a fresh child process
initialises a world-1 "nccl" group (RCCL on ROCm) before touching the GPU, decomposes two
matrices with the HIP engine through sharding.decompose_sharded, gathers the packed (codes, L,
R) payload to rank 0 over RCCL and checks it byte for byte against the direct results
(tests/rccl_child.py).  The world-2 logic of the same functions runs under gloo on the CPU
(tests/test_sharding_gloo.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(240)
def test_rccl_world1_gather_matches_direct_results():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_child.py")], env=env, capture_output=True,
                       text=True, timeout=200)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    rec = json.loads(lines[-1])
    print("rccl child:", rec)
    assert rec["backend"] == "nccl" and rec["world"] == 1 and rec["equal"] and rec["matrices"] == 2
