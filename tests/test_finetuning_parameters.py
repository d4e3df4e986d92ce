"""Finetuning parameter selection (reference ``tests/transformer/test_finetuning_parameter.py``): config
validation, the legacy ``use_seperate_lr_on_embeddings`` name, pattern matching across data-parallel ranks (a pattern
must match on SOME rank, checked collectively), exclusion patterns and first-match semantics."""
from __future__ import annotations

from types import SimpleNamespace

import pytest
import torch
from pydantic import ValidationError

from tests.dist_utils import run_distributed

pytestmark = pytest.mark.cpu


@pytest.mark.parametrize("cfg", [{}, {"finetune": True, "finetunable_parameters": ["a"], "parameters_exclude": ["b"]},
                                 {"finetune": True, "finetunable_parameters": ["a"]}])
def test_training_config_accepts(cfg):
    from scaling_amd.transformer.context.config import TrainingConfig

    TrainingConfig(**cfg)
    TrainingConfig.from_dict(cfg)


@pytest.mark.parametrize("cfg", [{"finetunable_parameters": ["a"]}, {"finetune": True},
                                 {"finetunable_parameters": ["a"], "parameters_exclude": ["b"]}])
def test_training_config_rejects(cfg):
    from scaling_amd.transformer.context.config import TrainingConfig

    with pytest.raises(ValidationError):
        TrainingConfig(**cfg)
    with pytest.raises(ValidationError):
        TrainingConfig.from_dict(cfg)


def test_legacy_field_name():
    from scaling_amd.transformer.context.config import TrainingConfig

    assert TrainingConfig(use_seperate_lr_on_embeddings=True).use_separate_lr_on_embeddings is True


def _npm(name: str):
    return (name, torch.tensor([1.0]), SimpleNamespace())


_PARAMS = {
    "unmatched": [[_npm("foo.not_relevant.bar"), _npm("foo.summarization.bar")],
                  [_npm("foo.summarization.bar"), _npm("foo.not_relevant_either.bar")]],
    "matched": [[_npm("foo.not_relevant.bar"), _npm("image_encoder.bar")],
                [_npm("foo.summarization.bar"), _npm("foo.not_relevant_either.bar")]],
    "excluded": [[_npm("foo.not_relevant.bar"), _npm("image_encoder.bar"), _npm("image_encoder.baz")],
                 [_npm("foo.summarization.bar"), _npm("foo.not_relevant_either.bar")]],
}


def _select(case: str):
    import torch.distributed as dist

    from scaling_amd.transformer.context.config import TrainingConfig
    from scaling_amd.transformer.model.model import _extract_parameters

    dist.init_process_group("gloo")
    rank = dist.get_rank()
    conf = TrainingConfig(finetune=True, finetunable_parameters=["summarization", "image_encoder"],
                          parameters_exclude=["image_encoder.baz"] if case == "excluded" else [])
    try:
        emb, no_wd, wd = _extract_parameters(conf, _PARAMS[case][rank])
        out = ("ok", [p[0] for p in emb], [p[0] for p in no_wd], [p[0] for p in wd])
    except ValueError as e:
        out = ("error", str(e))
    dist.destroy_process_group()
    return out


def test_unmatched_pattern_raises_on_every_rank():
    res = run_distributed(_select, 2, case="unmatched")
    for r in res.values():
        assert r[0] == "error" and "Unmatched finetunable parameters: {'image_encoder'}" in r[1]


@pytest.mark.parametrize("case", ["matched", "excluded"])
def test_patterns_matched_on_some_rank(case):
    res = run_distributed(_select, 2, case=case)
    assert res[0] == ("ok", [], [], ["image_encoder.bar"])
    assert res[1] == ("ok", [], [], ["foo.summarization.bar"])


@pytest.mark.parametrize("data,result", [(["foo", "bar", "foo.bar"], "foo"), (["baz", "bar", "bay.bar"], "bar"),
                                         (["baz", "buz", "bay.bar"], None), (["baz", "buz", "foo.bar"], "foo.bar")])
def test_find_matching_param_first_match(data, result):
    from scaling_amd.transformer.model.model import _find_matching_param

    assert _find_matching_param(_npm("foo.bar"), data) == result
