"""The multi-rank data path (all-gather of dictionary summaries, bitsets,
rare records, sizes; all-gather of plain sets; triangle row partition) on
one GPU: 2 and 3 ranks share the device through the host-staged transport,
and rank 0 checks every rank's rows bit-exactly against the CPU oracle
(cases in tests/mr_worker.py: bitset, sorted and sketch exchanges; a
C2-shaped collection with the complement-sparse words active on every
rank; a C4-shaped one). RCCL itself refuses two ranks on one device, so this is how the
exchange logic is exercised on a one-GPU box."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("world", [2, 3])
def test_multirank_host_transport(world):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(29600 + world), os.path.join(HERE, "mr_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert f"MULTIRANK_OK {world}" in r.stdout
    for case in ("base", "sparse", "c4"):
        assert f"CASE_OK {case} {world}" in r.stdout, case
