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


def _run(world, cases=None):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    if cases:
        env["MR_CASES"] = ",".join(cases)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(29600 + world), os.path.join(HERE, "mr_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert f"MULTIRANK_OK {world}" in r.stdout
    return r


@pytest.mark.parametrize("world", [2, 3])
def test_multirank_host_transport(world):
    r = _run(world)
    for case in ("base", "sparse", "c4"):
        assert f"CASE_OK {case} {world}" in r.stdout, case


def test_multirank_c4_eight_ranks():
    """C4's 8-GPU path at R = 8 — eight host-transport ranks
    sharing the GPU run the c4 case (the consuming code all-gather, the split
    build of the gathered collection with 8 shares of the code ranges and
    m = ceil(N / 8) sets each, its tier all-gathers, METHOD_AUTO on a
    replicated collection, the sorted join), every rank's rows bit-exact
    against the oracle (FastaDistanceProcessor.java:157-158)."""
    r = _run(8, ["c4"])
    assert "CASE_OK c4 8" in r.stdout
