"""Variable-length 3-12 s bucketed batching (BASELINE config 5), host side (CPU)."""
import torch

from nrse_amd import data as D


def _sampler(lengths, world=1, rank=0, seed=3, bs=4):
    edges = [int(s * 16000) for s in range(4, 13)]
    return D.LengthBucketBatchSampler(lengths, bs, edges, seed=seed, rank=rank, world=world)


def test_buckets_disjoint_and_homogeneous():
    ds = D.SyntheticVarLenPairs(203, 16000, 3.0, 12.0, [4, 8], seed=11)
    s = _sampler(ds.lengths)
    seen = set()
    for b in s:
        assert len(b) == 4
        ks = {s.bucket_of(ds.lengths[i]) for i in b}
        assert len(ks) == 1                          # one bucket per batch
        assert not (set(b) & seen)                   # an item at most once per epoch
        seen |= set(b)
    assert len(seen) > 0.8 * len(ds)                 # only bucket remainders are dropped


def test_epochs_and_ranks():
    ds = D.SyntheticVarLenPairs(160, 16000, 3.0, 12.0, [4, 8], seed=5)
    a0 = list(_sampler(ds.lengths))
    a1 = list(_sampler(ds.lengths))
    assert a0 == a1                                   # deterministic
    s = _sampler(ds.lengths)
    s.set_epoch(1)
    assert list(s) != a0                              # reshuffled per epoch
    r0 = list(_sampler(ds.lengths, world=2, rank=0))
    r1 = list(_sampler(ds.lengths, world=2, rank=1))
    assert len(r0) == len(r1) > 0
    assert not ({i for b in r0 for i in b} & {i for b in r1 for i in b})


def test_collate_pads_and_noise_lengths():
    ds = D.SyntheticVarLenPairs(8, 16000, 3.0, 12.0, [4, 8], seed=2)
    items = [ds[i] for i in range(4)]
    out = D.collate_varlen(items, 8000)
    L = out["clean"].shape[1]
    assert L % 8000 == 0 and L >= max(int(x) for x in out["lengths"])
    for i, it in enumerate(items):
        n = it["clean"].shape[0]
        assert torch.equal(out["clean"][i, :n], it["clean"]) and float(out["clean"][i, n:].abs().sum()) == 0.0
        assert int(out["noise_len"][i]) == it["noise"].shape[0]
    assert out["snr"].tolist() == [4, 8, 4, 8]


def test_loader_end_to_end():
    ds = D.SyntheticVarLenPairs(48, 16000, 3.0, 12.0, [4, 8], seed=9)
    dl = D.create_varlen_loader(ds, 4, num_workers=0)
    shapes = set()
    for batch in dl:
        shapes.add(batch["clean"].shape[1])
        assert batch["clean"].shape[0] == 4
    assert len(shapes) > 1                            # several step shapes over an epoch
