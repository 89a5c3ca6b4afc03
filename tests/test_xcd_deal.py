"""The XCD-aware deal of the traversal work queue (rt_hip.hip, trace_refill_kernel's fetch
loop, RT_XCD_CHUNK): the map (shard, j) -> group it uses, restated here, must hand out every
64-slot group exactly once over the 32 shards, in increasing order within a shard (a shard
is exhausted at its first group past the end), with every group of a chunk on the shards of
one XCD (shard % 8), and a block's shard sequence must visit all 32 shards, its own XCD's
four first.  The GPU parity tests check the kernel itself: a group handed out twice or never
would change the ray counts and the frame."""
import pytest

X, P, NFS = 8, 4, 32


def group_of(sh: int, j: int, xc: int) -> int:
    per = xc // P
    k = j // per
    return (k * X + sh % X) * xc + sh // X + (j % per) * P


def shard_seq(block: int):
    return [((block % X + sk // P) % X) + X * ((block // X + sk % P) % P) for sk in range(NFS)]


@pytest.mark.parametrize("xc", [4, 64, 512, 1 << 20])
@pytest.mark.parametrize("n_groups", [1, 5, 63, 64, 65, 1000, 4099])
def test_every_group_once(xc, n_groups):
    seen = []
    for sh in range(NFS):
        j, last = 0, -1
        while True:
            g = group_of(sh, j, xc)
            if g >= n_groups:
                break
            assert g > last  # increasing within a shard
            assert (g // xc) % X == sh % X  # the chunk's XCD owns the shard
            last = g
            seen.append(g)
            j += 1
    assert sorted(seen) == list(range(n_groups))


def test_block_visits_every_shard_own_xcd_first():
    for b in range(0, 2048, 7):
        seq = shard_seq(b)
        assert sorted(seq) == list(range(NFS))
        assert all(s % X == b % X for s in seq[:P])
        assert seq[0] % X == b % X  # blocks start on a shard of their own XCD (block b on XCD b % 8)
