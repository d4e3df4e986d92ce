"""Data pipeline: memory maps, item index parity with the reference's cached index, legacy MMIDIDX,
blended sampling, data loader order / resume / data-parallel sharding, finetuning datasets.
(Reference: tests/core/test_data/*, tests/transformer/test_data.py, test_blended_dataset.py.)"""
import json
import shutil
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.cpu
REF = Path("/root/reference/tests/transformer/files")


def _mmap(tmp: Path, docs: list) -> Path:
    from scaling_amd.core import MemoryMapDatasetBuilder

    with MemoryMapDatasetBuilder(tmp / "data") as b:
        for d in docs:
            b.add(np.array(d))
    return tmp / "data"


def test_memory_map_roundtrip_and_file_dataset(tmp_path):
    from scaling_amd.core import FileDataset, MemoryMapDataset

    rng = np.random.RandomState(0)
    docs = [rng.randint(0, 30000, size=rng.randint(1, 50)) for _ in range(40)]
    prefix = _mmap(tmp_path, docs)
    for mm in (MemoryMapDataset(prefix), MemoryMapDataset(prefix, load_index_to_memory=True), FileDataset(prefix)):
        assert len(mm) == 40
        for i in (0, 7, 39):
            np.testing.assert_array_equal(np.asarray(mm[i]), docs[i])
        np.testing.assert_array_equal(np.asarray(mm.sizes()), [len(d) for d in docs])


def _reference_text_index(sizes, order, seq, only_full=False, every_n=0):
    """The reference packing loop (text_dataset.py:223-335), transcribed as the spec."""
    items, cur, tok, full, half, in_half = [], [], 0, 0, 0, False
    for doc in order:
        pos, cnt = 0, sizes[doc]
        while pos < cnt - 1:
            end = min(cnt, pos + 1 + seq - tok)
            if only_full:
                if in_half:
                    pass
                elif end - pos < seq + 1:
                    if every_n != 0 and (full / every_n - half) >= 1:
                        in_half = True
                    else:
                        break
                else:
                    full += 1
            tok += end - pos
            cur.append((doc, pos, end))
            if tok == seq + 1:
                items.append(cur)
                cur, tok = [], 0
                if in_half:
                    half += 1
                in_half = False
            pos = end - 1
    return items


@pytest.mark.parametrize("seq,only_full,every_n", [(8, False, 0), (64, False, 0), (16, True, 0), (16, True, 4), (4, True, 256)])
def test_native_text_index_matches_reference_algorithm(seq, only_full, every_n):
    from scaling_amd import _data

    rng = np.random.RandomState(3)
    sizes = rng.randint(1, 120, size=300).astype(np.int64)
    order = np.arange(300)
    rng.shuffle(order)
    flat, pairs = _data.text_index(sizes, order.astype(np.int64), seq, only_full, every_n)
    ref = _reference_text_index(sizes.tolist(), order.tolist(), seq, only_full, every_n)
    got = [flat[s : s + n].reshape(-1, 3).tolist() for s, n in pairs.reshape(-1, 2)]
    assert got == [[list(t) for t in item] for item in ref]


@pytest.mark.skipif(not (REF / "dataset" / "data.bin").exists(), reason="reference fixtures not mounted")
def test_text_dataset_index_bit_identical_to_reference_cache(tmp_path):
    from scaling_amd.transformer.data import TextDataset

    for f in ("data.bin", "data.idx", "data.meta.json"):
        shutil.copy(REF / "dataset" / f, tmp_path / f)
    ds = TextDataset(data_prefix=tmp_path / "data", sequence_length=64, seed=42)
    stem = "data_index_cache_decoder_dataset_seed_42_seq_len_64"
    for suffix in (".bin", ".idx"):
        mine = np.fromfile(tmp_path / (stem + suffix), dtype=np.int64)
        ref = np.fromfile(REF / "dataset" / (stem + suffix), dtype=np.int64)
        np.testing.assert_array_equal(mine, ref)
    assert json.loads((tmp_path / (stem + ".meta.json")).read_text())["document_count"] == len(ds) == 55
    for i in range(len(ds)):
        assert ds[i].token_ids.shape == (65,)
    batch = TextDataset.sync_batch_to_model_parallel(None, ds.collate([ds[0], ds[1]]))
    assert batch.input_token_ids.shape == (2, 64) and batch.target_token_ids.shape == (2, 64)
    assert torch.equal(batch.input_token_ids[:, 1:], batch.target_token_ids[:, :-1])


@pytest.mark.skipif(not (REF / "dataset" / "legacy").exists(), reason="reference fixtures not mounted")
def test_legacy_dataset_and_blend(tmp_path):
    from scaling_amd.core import BlendedDatasetConfig
    from scaling_amd.transformer.data import LegacyBlendedDataset, TextDataset
    from scaling_amd.transformer.data.legacy_dataset import MMapIndexedDataset

    for f in ("enron_text_document_100.bin", "enron_text_document_100.idx"):
        shutil.copy(REF / "dataset" / "legacy" / f, tmp_path / f)
    raw = MMapIndexedDataset(str(tmp_path / "enron_text_document_100"))
    assert len(raw) == 100
    ds = TextDataset(data_prefix=tmp_path / "enron_text_document_100", sequence_length=32, seed=7, legacy_dataset=True)
    assert (tmp_path / "enron_text_document_100_index_cache_decoder_dataset_seed_7_seq_len_32.done").is_file()
    assert len(ds) > 0 and all(ds[i].token_ids.shape == (33,) for i in range(min(len(ds), 20)))
    # every item is a concatenation of consecutive document slices
    item = np.asarray(ds.data_item_index[0]).reshape(-1, 3)
    toks = np.concatenate([raw[int(d)][int(a):int(b)] for d, a, b in item])
    np.testing.assert_array_equal(ds[0].token_ids.numpy(), toks)
    ds2 = TextDataset(data_prefix=tmp_path / "enron_text_document_100", sequence_length=16, seed=7, legacy_dataset=True)
    blend = LegacyBlendedDataset(seed=7, config=BlendedDatasetConfig(cache_directory=tmp_path), datasets=[ds, ds2])
    assert len(blend) > 0
    blend[0]
    blend[len(blend) - 1]


def test_legacy_blend_stops_at_first_completed_quota():
    from scaling_amd.transformer.data.legacy_blended_dataset import legacy_blend

    rows = legacy_blend(np.array([4, 2, 8]))
    counts = np.bincount(rows[:, 0], minlength=3)
    assert counts[1] == 2 and counts[0] <= 4 and counts[2] <= 8
    for d in range(3):  # indices per dataset are consecutive from 0
        np.testing.assert_array_equal(rows[rows[:, 0] == d][:, 1], np.arange(counts[d]))


def _python_blend(counts):
    sampled = np.zeros(len(counts), dtype=np.int64)
    out = []
    while (sampled < counts).any():
        ratio = np.where(sampled < counts, sampled / counts, np.inf)
        i = int(ratio.argmin())
        out.append((i, sampled[i]))
        sampled[i] += 1
    return np.array(out)


def test_native_blended_sample_matches_python(tmp_path):
    from scaling_amd.core.data.blended_dataset import native_blended_sample

    counts = np.array([7, 3, 11, 1])
    n = native_blended_sample(counts, str(tmp_path / "blend"))
    got = np.fromfile(tmp_path / "blend.bin", dtype=np.int64).reshape(-1, 2)
    assert n == counts.sum()
    np.testing.assert_array_equal(got, _python_blend(counts))


class _Range:
    pass


def _range_dataset(n):
    from scaling_amd.core import BaseDataset, BaseDatasetItem

    class Item(BaseDatasetItem):
        def __init__(self, v):
            self.v = v

    class DS(BaseDataset):
        def __init__(self):
            super().__init__(seed=0)

        def ident(self):
            return "range"

        def __len__(self):
            return n

        def __getitem__(self, i):
            return Item(i)

        def set_seed(self, seed, shuffle=True):
            self.seed = seed

        def collate(self, batch):
            return torch.tensor([b.v for b in batch])

        @staticmethod
        def sync_batch_to_model_parallel(topology, batch):
            return batch

    return DS()


class _Topo:
    def __init__(self, dp, rank, mbs):
        from scaling_amd.core import TopologyConfig

        self.config = TopologyConfig(global_rank=0, world_size=dp, model_parallel_size=1, pipe_parallel_size=1,
                                     data_parallel_size=dp, micro_batch_size=mbs, gradient_accumulation_steps=1)
        self.data_parallel_rank = rank


def test_dataloader_sharding_and_resume():
    from scaling_amd.core import DataLoader

    ds = _range_dataset(40)
    seen = []
    for r in range(2):
        dl = DataLoader(seed=1, consumed_samples=0, dataset=ds, topology=_Topo(2, r, 4))
        seen.append(torch.cat([next(dl) for _ in range(5)]).tolist())
    assert set(seen[0]).isdisjoint(seen[1]) and len(set(seen[0]) | set(seen[1])) == 40
    # resume after 3 global batches (3 * mbs * dp samples) continues exactly
    dl = DataLoader(seed=1, consumed_samples=3 * 4 * 2, dataset=ds, topology=_Topo(2, 0, 4))
    assert torch.cat([next(dl) for _ in range(2)]).tolist() == seen[0][12:20]


@pytest.mark.skipif(not (REF / "llama2-tokenizer.json").exists(), reason="reference tokenizer not mounted")
def test_finetuning_datasets(tmp_path):
    from scaling_amd.transformer.data import FinetuningChatDataset, FinetuningTextDataset
    from scaling_amd.transformer.tokenizer import load_tokenizers

    tok, tok_nps = load_tokenizers(REF / "llama2-tokenizer.json")
    ds = FinetuningTextDataset(data_prefix=REF / "dataset" / "finetuning.json", sequence_length=32, seed=1,
                               softprompt_n_tokens=2, tokenizer=tok, tokenizer_no_prefix_space=tok_nps)
    it = ds[0]
    assert it.input_token_ids.shape == (32,) and it.loss_weights.shape == (32,)
    assert it.loss_weights.sum() > 0
    batch = FinetuningTextDataset.sync_batch_to_model_parallel(None, ds.collate([ds[0], ds[1]]))
    assert batch.loss_weights.shape == (2, 32)
    # memory-map variant via convert_jsonl
    FinetuningTextDataset.convert_jsonl(REF / "dataset" / "finetuning.jsonl", tok, tok_nps, tmp_path / "ft")
    ds_mm = FinetuningTextDataset(data_prefix=tmp_path / "ft", sequence_length=32, seed=1, softprompt_n_tokens=0,
                                  tokenizer=tok, tokenizer_no_prefix_space=tok_nps, memory_map_dataset=True)
    assert len(ds_mm) > 0 and ds_mm[0].input_token_ids.shape == (32,)
    chat = FinetuningChatDataset(data_path=REF / "dataset" / "finetuning_chat.jsonl", sequence_length=64, seed=1,
                                 softprompt_n_tokens=0, tokenizer=tok, tokenizer_no_prefix_space=tok_nps)
    c = chat[0]
    assert c.input_token_ids.shape == (64,) and 0 < c.loss_weights.sum() < 64
