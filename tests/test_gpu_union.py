"""The engine group's device key union (spanagg_union.hip sa::key_union,
reached through the sa_key_union_probe diagnostic): the sorted distinct
non-zero series ids of the members' gathered key lists, the dense index of
the group flush (standing in for the one collector
instance at /root/reference/docker-compose.yml:748-756).  Checked bit-exactly
against numpy's unique on the same ids: hash-like ids with every member's
list repeated, the zero padding RCCL's all-gather adds, ragged sizes around
the bucket geometry, and a skewed id set whose single bucket is far above
the LDS sort's 8,192 ids (the global-scratch network)."""
import numpy as np
import pytest

from spanagg import Config, Engine

pytestmark = pytest.mark.gpu


def _ref(ids):
    u = np.unique(np.asarray(ids, dtype=np.uint64))
    return u[u != 0]


@pytest.fixture(scope="module")
def eng():
    with Engine(Config(n_services=1, n_windows=16)) as e:
        yield e


@pytest.mark.parametrize("n", [1, 2, 1023, 1024, 1025, 65_537, 1_000_003])
def test_union_of_hash_ids(eng, n):
    rng = np.random.Generator(np.random.PCG64(n))
    ids = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    assert np.array_equal(eng.key_union_probe(ids), _ref(ids))


def test_union_of_8_members_with_padding(eng):
    """8 members' lists of ~750 k ids drawn from 1 M series (each id in several
    lists), zero-padded to the longest list as the all-gather pads them."""
    rng = np.random.Generator(np.random.PCG64(8))
    series = rng.integers(1, 2**64 - 1, 1_000_000, dtype=np.uint64)
    lists = [series[rng.random(len(series)) < 0.75] for _ in range(8)]
    nmax = max(len(x) for x in lists)
    gathered = np.concatenate([np.concatenate([x, np.zeros(nmax - len(x), np.uint64)]) for x in lists])
    got = eng.key_union_probe(gathered)
    assert np.array_equal(got, _ref(gathered))
    assert len(got) == len(np.unique(np.concatenate(lists)))


def test_union_edge_values(eng):
    ids = np.array([0, 0, 2**64 - 1, 1, 2**64 - 1, 2**63, 1, 0, 2**63 - 1], dtype=np.uint64)
    assert np.array_equal(eng.key_union_probe(ids), _ref(ids))
    assert len(eng.key_union_probe(np.zeros(5000, np.uint64))) == 0


def test_union_oversized_bucket_takes_the_global_network(eng):
    """30,000 distinct ids sharing their top 20 bits land in one bucket (more
    than the 8,192 one workgroup sorts in LDS), beside uniform ids."""
    rng = np.random.Generator(np.random.PCG64(3))
    skew = (np.uint64(0xABCDE) << np.uint64(44)) | rng.integers(0, 2**44, 30_000, dtype=np.uint64)
    ids = np.concatenate([skew, skew[:5000], rng.integers(1, 2**64 - 1, 100_000, dtype=np.uint64)])
    rng.shuffle(ids)
    assert np.array_equal(eng.key_union_probe(ids), _ref(ids))


def test_union_of_ragged_members_mostly_padding(eng):
    """Members whose key counts differ widely (one holds 1 M ids, seven hold
    10 k): the all-gather's zero padding is ~7 M ids, 87 % of the input.  The
    zeros are neither counted nor placed, so no bucket overflows into the
    global-scratch network (advisor r4: they used to pile into bucket 0)."""
    rng = np.random.Generator(np.random.PCG64(12))
    big = rng.integers(1, 2**64 - 1, 1_000_000, dtype=np.uint64)
    lists = [big] + [rng.choice(big, 10_000, replace=False) for _ in range(7)]
    nmax = max(len(x) for x in lists)
    gathered = np.concatenate([np.concatenate([x, np.zeros(nmax - len(x), np.uint64)]) for x in lists])
    assert (gathered == 0).mean() > 0.8
    assert np.array_equal(eng.key_union_probe(gathered), _ref(gathered))
