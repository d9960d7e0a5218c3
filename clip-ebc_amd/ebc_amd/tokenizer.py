"""CLIP byte-level BPE tokenizer: `SimpleTokenizer` and `tokenize` (models/clip/_clip/simple_tokenizer.py:62,
models/clip/_clip/utils.py:209-249).  Init-only host code: it turns the bin prompts into token ids once,
at model construction (models/clip/model.py:109-115); nothing here runs per step.

The algorithm is CLIP's published one: text -> ftfy/html clean-up, whitespace collapse, lower case ->
regex pre-tokenisation -> each piece's UTF-8 bytes mapped to printable code points -> greedy merging of
the lowest-ranked adjacent pair (the last symbol of a word carries the end-of-word mark "</w>") -> ids.
Vocabulary: the 256 byte symbols, the same with "</w>", one symbol per merge, then <|startoftext|> and
<|endoftext|> (49408 ids).  The merge list is data (`data/clip_bpe_merges.txt.gz`: the 48894 merges CLIP
uses, extracted from the reference's bpe_simple_vocab_16e6.txt.gz by tests/golden/make_golden.py); pass
`bpe_path` to use another merges file (the full vocab file works too: only its first 48894 merges are
read).  `ftfy` is not installed here: without it the clean-up is html.unescape only, which leaves ASCII
prompts unchanged.
"""
from __future__ import annotations

import gzip
import html
import os
from typing import Dict, List, Sequence, Tuple, Union

import regex
import torch

N_MERGES = 49152 - 256 - 2          # CLIP uses this many merges (vocab 49408 = 2*256 + merges + 2 specials)
DEFAULT_BPE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "clip_bpe_merges.txt.gz")
SOT, EOT = "<|startoftext|>", "<|endoftext|>"
_PIECES = regex.compile(r"<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+",
                        regex.IGNORECASE)

try:                                                      # optional, as in the reference's requirements
    import ftfy as _ftfy
except ImportError:                                       # pragma: no cover - absent in this image
    _ftfy = None


def byte_symbols() -> Dict[int, str]:
    """Each byte -> a printable code point: the printable Latin-1 bytes map to themselves, the other 68
    to 256, 257, ... in byte order (the order fixes the first 256 vocabulary ids)."""
    table = {b: chr(b) for b in [*range(33, 127), *range(161, 173), *range(174, 256)]}
    nxt = 256
    for b in range(256):
        if b not in table:
            table[b] = chr(nxt)
            nxt += 1
    return table


def clean(text: str) -> str:
    if _ftfy is not None:
        text = _ftfy.fix_text(text)
    text = html.unescape(html.unescape(text)).strip()
    return regex.sub(r"\s+", " ", text).strip()          # collapse whitespace runs


class SimpleTokenizer:
    """Byte-level BPE with CLIP's vocabulary (simple_tokenizer.py:62)."""

    def __init__(self, bpe_path: str = DEFAULT_BPE):
        if not os.path.exists(bpe_path):
            raise FileNotFoundError(f"CLIP BPE merges not found at {bpe_path}")
        with gzip.open(bpe_path, "rt", encoding="utf-8") as f:
            lines = f.read().split("\n")
        if lines and lines[0].startswith("#"):           # the original vocab file starts with a version line
            lines = lines[1:]
        merges = [tuple(l.split()) for l in lines[:N_MERGES]]
        if len(merges) != N_MERGES or any(len(m) != 2 for m in merges):
            raise ValueError(f"{bpe_path}: expected {N_MERGES} merge lines")
        self.byte_encoder = byte_symbols()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        syms = list(self.byte_encoder.values())
        vocab = syms + [s + "</w>" for s in syms] + ["".join(m) for m in merges] + [SOT, EOT]
        self.encoder = {s: i for i, s in enumerate(vocab)}
        self.decoder = {i: s for s, i in self.encoder.items()}
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.cache = {SOT: SOT, EOT: EOT}

    def bpe(self, piece: str) -> str:
        if piece in self.cache:
            return self.cache[piece]
        word: List[str] = list(piece[:-1]) + [piece[-1] + "</w>"]
        while len(word) > 1:
            ranked = [(self.bpe_ranks.get((a, b), None), i) for i, (a, b) in enumerate(zip(word, word[1:]))]
            ranked = [(r, i) for r, i in ranked if r is not None]
            if not ranked:
                break
            best = min(ranked)[0]
            a, b = next((word[i], word[i + 1]) for r, i in ranked if r == best)
            merged, i = [], 0
            while i < len(word):                          # merge every occurrence of the pair, left to right
                if i + 1 < len(word) and word[i] == a and word[i + 1] == b:
                    merged.append(a + b)
                    i += 2
                else:
                    merged.append(word[i])
                    i += 1
            word = merged
        out = " ".join(word)
        self.cache[piece] = out
        return out

    def encode(self, text: str) -> List[int]:
        ids: List[int] = []
        for piece in _PIECES.findall(clean(text).lower()):
            sym = "".join(self.byte_encoder[b] for b in piece.encode("utf-8"))
            ids.extend(self.encoder[t] for t in self.bpe(sym).split(" "))
        return ids

    def decode(self, ids: Sequence[int]) -> str:
        syms = "".join(self.decoder[int(i)] for i in ids)
        # "</w>" is made of printable bytes that map to themselves: decode first, then mark word ends
        return bytearray(self.byte_decoder[c] for c in syms).decode("utf-8", errors="replace").replace("</w>", " ")


_DEFAULT: Dict[str, SimpleTokenizer] = {}


def _tokenizer(bpe_path: str = DEFAULT_BPE) -> SimpleTokenizer:
    if bpe_path not in _DEFAULT:
        _DEFAULT[bpe_path] = SimpleTokenizer(bpe_path)
    return _DEFAULT[bpe_path]


def tokenize(texts: Union[str, List[str]], context_length: int = 77, truncate: bool = False,
             bpe_path: str = DEFAULT_BPE) -> torch.IntTensor:
    """models/clip/_clip/utils.py:209-249: [n, context_length] int32 ids, <sot> text <eot> zero-padded; a text
    longer than the context raises RuntimeError unless `truncate` (then the last kept id becomes <eot>)."""
    if isinstance(texts, str):
        texts = [texts]
    tok = _tokenizer(bpe_path)
    sot, eot = tok.encoder[SOT], tok.encoder[EOT]
    out = torch.zeros(len(texts), context_length, dtype=torch.int)
    for i, t in enumerate(texts):
        ids = [sot] + tok.encode(t) + [eot]
        if len(ids) > context_length:
            if not truncate:
                raise RuntimeError(f"Input {t} is too long for context length {context_length}")
            ids = ids[:context_length]
            ids[-1] = eot
        out[i, :len(ids)] = torch.tensor(ids, dtype=torch.int)
    return out
