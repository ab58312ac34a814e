"""RCCL on hardware: ncclCommInitRank and ncclAllGather
(gdist_api.hip, gdist_comm_init / allgather) run on the one-GPU box through a
one-rank communicator that is forced through every exchange (option
force_exchange), in a subprocess with its own time limit."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_rccl_one_rank_exchange():
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_worker.py")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "RCCL_OK" in r.stdout
