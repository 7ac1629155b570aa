"""CLIP byte-level BPE tokenizer.

Reproduces the token ids of ``transformers.CLIPTokenizer`` on ``openai/clip-vit-large-patch14``
(used by the reference at ``comfy/sd1_clip.py:360``) without transformers: vocabulary is derived
from the merge list (256 byte symbols, the same with ``</w>``, one symbol per merge, then the two
special tokens — 49408 ids). The hot loop (BPE merge per word) runs in the C++ runtime
(``csrc/runtime/bpe.cpp``) when it is built; this module is the pure-Python fallback / oracle.
"""
from __future__ import annotations

import functools
import gzip
import html
import os

import regex as re

from .. import _native

_DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "clip_bpe_merges.txt.gz")

_PAT = re.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""",
                  re.IGNORECASE)


def bytes_to_unicode():
    """The reversible byte -> printable-unicode map used by GPT-2/CLIP BPE."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def _clean(text: str) -> str:
    text = html.unescape(html.unescape(text))
    text = " ".join(text.split())
    return text.strip().lower()


class CLIPTokenizer:
    BOS = 49406
    EOS = 49407

    def __init__(self, merges_path: str = _DATA):
        with gzip.open(merges_path, "rt", encoding="utf-8") as f:
            merges = [tuple(l.split()) for l in f.read().split("\n") if l.strip()]
        self.byte_encoder = bytes_to_unicode()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        vocab = list(self.byte_encoder.values())
        vocab = vocab + [v + "</w>" for v in vocab]
        for m in merges:
            vocab.append("".join(m))
        vocab.extend(["<|startoftext|>", "<|endoftext|>"])
        self.encoder = {v: i for i, v in enumerate(vocab)}
        self.decoder = {i: v for v, i in self.encoder.items()}
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self._native = None
        rt = _native.load_runtime()
        if rt is not None and hasattr(rt, "BPE"):
            try:
                self._native = rt.BPE(["{} {}".format(*m) for m in merges], vocab)
            except Exception:  # pragma: no cover
                self._native = None

    @functools.lru_cache(maxsize=65536)
    def _bpe(self, token: str) -> tuple:
        word = tuple(token[:-1]) + (token[-1] + "</w>",)
        if len(word) == 1:
            return word
        while True:
            best = None
            best_rank = None
            for i in range(len(word) - 1):
                r = self.bpe_ranks.get((word[i], word[i + 1]))
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = i, r
            if best is None:
                break
            a, b = word[best], word[best + 1]
            new = []
            i = 0
            while i < len(word):
                if i < len(word) - 1 and word[i] == a and word[i + 1] == b:
                    new.append(a + b)
                    i += 2
                else:
                    new.append(word[i])
                    i += 1
            word = tuple(new)
            if len(word) == 1:
                break
        return word

    def encode(self, text: str) -> list[int]:
        """Token ids WITHOUT BOS/EOS."""
        text = _clean(text)
        ids = []
        for tok in _PAT.findall(text):
            if tok == "<|startoftext|>":
                ids.append(self.BOS)
                continue
            if tok == "<|endoftext|>":
                ids.append(self.EOS)
                continue
            u = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            if self._native is not None:
                ids.extend(self._native.encode_word(u))
            else:
                ids.extend(self.encoder[p] for p in self._bpe(u))
        return ids

    def __call__(self, text: str) -> dict:
        return {"input_ids": [self.BOS] + self.encode(text) + [self.EOS]}

    def decode(self, ids) -> str:
        s = "".join(self.decoder.get(int(i), "") for i in ids)
        b = bytearray(self.byte_decoder[c] for c in s if c in self.byte_decoder)
        return b.decode("utf-8", errors="replace").replace("</w>", " ")

    def get_vocab(self):
        return dict(self.encoder)


@functools.lru_cache(maxsize=1)
def get_clip_tokenizer() -> CLIPTokenizer:
    return CLIPTokenizer()
