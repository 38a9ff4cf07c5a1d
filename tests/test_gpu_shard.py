"""HIP stable pack by owning rank (sg_shard_pack / sg_shard_unpack) against a numpy
restatement of the same partition: owner = key % world, local key = key // world, arrival order
kept per destination, destinations in rank order."""
import importlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")
sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
reshard = importlib.import_module("siddhi-1_amd.reshard")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,n", [(1, 1000), (2, 12345), (3, 70001), (8, 1 << 20), (7, 4096), (8, 1)])
def test_shard_pack_is_a_stable_partition(world, n):
    d = synth.stock_ticks(3 * n, n, 1 << 16)
    dev = torch.device("cuda", 0)
    cols = {"key": torch.from_numpy(d["key"].view(np.int32)).to(dev), "ts": torch.from_numpy(d["ts"]).to(dev),
            "price": torch.from_numpy(d["price"]).to(dev), "volume": torch.from_numpy(d["volume"]).to(dev)}
    g = reshard.reshard_device(sa.load_hip_library(), cols, world, exchange=False)  # the packed rows
    torch.cuda.synchronize()
    own = d["key"] % world
    order = np.argsort(own, kind="stable")
    assert np.array_equal(g["key"].cpu().numpy().view(np.uint32), (d["key"] // world)[order])
    assert np.array_equal(g["ts"].cpu().numpy(), d["ts"][order])
    assert np.array_equal(g["price"].cpu().numpy(), d["price"][order])
    assert np.array_equal(g["volume"].cpu().numpy(), d["volume"][order])
