"""Two ranks on two GPUs over RCCL (skipped on a one-GPU box): libkwmatch's kw_allgather_hits with root 0 and
root -1, and the drop-in's --gpus 2 main path against the reference's outputs (tests/multi_gpu_worker.py,
started by torch.distributed.run with one process per GPU)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_rccl_exchange_and_main(tmp_path):
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip('needs two GPUs')
    from tests import golden_data
    (tmp_path / 'articles.csv').write_bytes(golden_data.articles_csv_bytes())
    with socket.socket() as so:
        so.bind(('127.0.0.1', 0))
        port = so.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2', '--master-addr',
           '127.0.0.1', f'--master-port={port}', os.path.join(REPO, 'tests', 'multi_gpu_worker.py'), str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert 'multi-GPU ok 2' in r.stdout
