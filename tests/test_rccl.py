"""RCCL on the GPU: a one-rank `nccl` process group on the MI355X round-trips the data-plane
collectives (stats all_reduce, size all_gather + bitstream gather, frame scatter) — the same
code the N-rank bench and node_job run."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def rccl_world1():
    import torch
    import torch.distributed as dist

    from thinvids_amd.parallel.launch import free_port

    old = {k: os.environ.get(k) for k in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE")}
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    yield dev
    dist.destroy_process_group()
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def test_rccl_world1_collectives(rccl_world1):
    import torch

    from thinvids_amd.parallel.comm import allreduce_stats, gather_bytes_to_root, scatter_frames_from_root

    dev = rccl_world1
    s = allreduce_stats([1.5, 2.5, 1e9], dev)
    np.testing.assert_array_equal(s, [1.5, 2.5, 1e9])
    m = allreduce_stats([3.0, 4.0], dev, op="max")
    np.testing.assert_array_equal(m, [3.0, 4.0])
    payload = bytes(range(256)) * 1000
    g = gather_bytes_to_root(payload, dev)
    assert g == [payload]
    frames = np.arange(2 * 4096, dtype=np.uint8).reshape(2, 4096)
    out = scatter_frames_from_root([frames], frames.shape, dev)
    assert out.is_cuda and torch.equal(out.cpu(), torch.from_numpy(frames))


def test_rccl_world1_node_job_allreduce_path(rccl_world1, tmp_path):
    """node_job's 2-pass RC statistics all-reduce runs through RCCL on the device."""
    import torch

    from thinvids_amd.parallel.comm import allreduce_stats

    x = torch.arange(64, dtype=torch.float64)
    got = allreduce_stats(x.numpy(), rccl_world1)
    np.testing.assert_array_equal(got, x.numpy())
