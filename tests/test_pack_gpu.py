"""The halo pack, dl_step_rows_tiled_peers (csrc/aux_kernels.hip step_rows_tiled_kernel): every
peer's send block [tiles, n_b, T] = x - lr*g of its rows, in one launch.  Checked bit for bit
against numpy float32 (two roundings: fl(x - fl(lr*g)), as the fused round's local step) over
the kernel's lane-group shapes -- one tile's lanes (rows x T/4) below a wave, between a wave and
256 (several lane groups per workgroup), and above 256 (several workgroups per tile) -- and tile
counts that leave ragged runs."""
import numpy as np
import pytest
import torch

from distributed_learning_amd import engine

pytestmark = pytest.mark.gpu


def _case(cuda, T, sizes, tiles, n_rows, with_g, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((tiles, n_rows, T)).astype(np.float32)
    g = rng.standard_normal((tiles, n_rows, T)).astype(np.float32)
    sel = rng.permutation(n_rows)[:sum(sizes)].astype(np.int32)
    row0 = [0] + list(np.cumsum(sizes))
    lr = np.float32(0.0125)
    X = torch.from_numpy(x).to(cuda)
    G = torch.from_numpy(g).to(cuda) if with_g else None
    outs = [torch.full((tiles, n, T), float("nan"), device=cuda) for n in sizes]
    engine.step_rows_tiled_peers(X, torch.from_numpy(sel).to(cuda), row0, outs, G=G,
                                 lr=float(lr))
    torch.cuda.synchronize()
    want = x[:, sel, :] - lr * g[:, sel, :] if with_g else x[:, sel, :]
    for b, o in enumerate(outs):
        got = o.cpu().numpy()
        exp = want[:, row0[b]:row0[b + 1], :]
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), (T, sizes, b)


@pytest.mark.parametrize("T", [4, 16, 64])
@pytest.mark.parametrize("sizes", [[1], [3, 5], [32, 32, 32], [7, 70, 1, 100], [200, 150],
                                   [5] * 16])
def test_pack_matches_numpy(cuda, T, sizes):
    _case(cuda, T, sizes, tiles=37, n_rows=400, with_g=True, seed=T * 100 + len(sizes))


@pytest.mark.parametrize("tiles", [1, 3, 8, 65, 1031])
def test_pack_ragged_tile_runs(cuda, tiles):
    # 96 rows at T = 16: 96 lanes per tile -> two 128-lane groups per workgroup
    _case(cuda, 16, [32, 32, 32], tiles=tiles, n_rows=128, with_g=True, seed=tiles)


def test_pack_without_gradient(cuda):
    _case(cuda, 16, [10, 20], tiles=50, n_rows=64, with_g=False, seed=7)
