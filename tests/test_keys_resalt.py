"""Series-id re-salting (SURVEY.md 7 'Key identity quirks'): a 64-bit id
collision between two distinct (resource, key) pairs never throws; the later
one takes the next seed.  The connector's ConsumeTraces never fails."""
from spanagg import keys


def test_collision_is_resalted(monkeypatch):
    real = keys.series_hash_seeded
    monkeypatch.setattr(keys, "series_hash_seeded", lambda rh, k, seed: 42 if seed == 0 else real(rh, k, seed))
    d = keys.KeyDictionary()
    a = d.intern(1, b"a", {}, {})
    b = d.intern(1, b"b", {}, {})
    c = d.intern(2, b"a", {}, {})
    assert a == 42 and len({a, b, c}) == 3 and 0 not in (a, b, c)
    assert d.collisions == 2
    assert d.intern(1, b"b", {}, {}) == b and d.collisions == 2  # stable, counted once
    assert d[b][1] == b"b" and d[c][0] == 2


def test_zero_id_takes_the_next_seed(monkeypatch):
    real = keys.series_hash_seeded
    monkeypatch.setattr(keys, "series_hash_seeded", lambda rh, k, seed: 0 if seed == 0 else real(rh, k, seed))
    assert keys.series_hash(7, b"k") == real(7, b"k", 1)


def test_no_collision_keeps_seed_zero():
    d = keys.KeyDictionary()
    assert d.intern(3, b"x", {}, {}) == keys.series_hash_seeded(3, b"x", 0) == keys.series_hash(3, b"x")
    assert d.collisions == 0
