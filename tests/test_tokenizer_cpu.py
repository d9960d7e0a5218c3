"""CPU: the CLIP BPE tokenizer (ebc_amd/tokenizer.py) against the reference tokenizer's own outputs:
the F6 prompts, every standard count prompt of data/prompt_tokens.json, and F6b's assorted texts
(unicode, punctuation, html entities, contractions, whitespace runs, empty and overlong input)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import REPO, golden


def test_tokenizer_matches_reference_texts():
    from ebc_amd.tokenizer import SimpleTokenizer
    tok = SimpleTokenizer()
    d = golden("f6b_tokens.npz")
    offs = d["offsets"]
    for i, t in enumerate(d["texts"]):
        assert tok.encode(str(t)) == d["ids"][offs[i]:offs[i + 1]].tolist(), str(t)


def test_tokenize_matches_f6_and_the_prompt_table():
    from ebc_amd.tokenizer import tokenize
    d = golden("f6_text.npz")
    np.testing.assert_array_equal(tokenize([str(p) for p in d["prompts_word"]]).numpy(), d["tokens_word"])
    np.testing.assert_array_equal(tokenize([str(p) for p in d["prompts_number"]]).numpy(), d["tokens_number"])
    with open(os.path.join(REPO, "clip-ebc_amd", "ebc_amd", "data", "prompt_tokens.json")) as f:
        table = json.load(f)
    prompts = sorted(table)
    toks = tokenize(prompts)
    for i, p in enumerate(prompts):
        ids = table[p]
        assert toks[i, :len(ids)].tolist() == ids and not toks[i, len(ids):].any(), p


def test_tokenize_context_and_truncate():
    from ebc_amd.tokenizer import tokenize, SimpleTokenizer
    long = "a " * 100
    with pytest.raises(RuntimeError):
        tokenize(long)
    t = tokenize(long, truncate=True)
    tok = SimpleTokenizer()
    assert t.shape == (1, 77) and t.dtype == torch.int32
    assert int(t[0, 0]) == tok.encoder["<|startoftext|>"] and int(t[0, 76]) == tok.encoder["<|endoftext|>"]
    assert tok.decode(tok.encode("There are twenty people.")).strip() == "there are twenty people ."


def test_prompt_tokens_outside_the_table():
    """Any prompt now tokenizes (round 1 raised KeyError outside the standard table)."""
    from ebc_amd.text import format_count, prompt_tokens
    from ebc_amd.tokenizer import tokenize
    p = format_count((5.0, 9.0), "word")
    np.testing.assert_array_equal(prompt_tokens([p]).numpy(), tokenize([p]).numpy())
