"""Prompt -> conditioning: emphasis parsing, 77-token chunking, textual inversion, clip-skip,
weighted interpolation, and the SD1 / SD2 / SDXL / SDXL-refiner / Stable-Cascade encoder stacks.

Behavioural parity with ``comfy/sd1_clip.py`` (``parse_parentheses``/``token_weights`` :201-247,
``SDTokenizer.tokenize_with_weights`` :398-480 incl. max_word_length=8 word splitting,
``ClipTokenWeightEncoder.encode_token_weights`` :26-60 weighted interpolation against the empty
prompt, ``SDClipModel.forward`` layer selection :162-193), ``sd2_clip.py``, ``sdxl_clip.py``
(L‖G hidden concat, G pooled) and the Cascade G encoder.

Differences by design: the weighted interpolation ``z = (z - z_empty) * w + z_empty`` is one
vectorised op over a weight tensor (the reference loops per token in Python), and every chunk
of every prompt is encoded in ONE batched transformer call.
"""
from __future__ import annotations

import logging
import os

import torch

from ..runtime import device as dm

from ..runtime.tokenizer import get_clip_tokenizer
from .clip import CLIPTextModel, CLIP_L_CONFIG, CLIP_G_CONFIG, CLIP_H_CONFIG


# ------------------------------------------------------------------------------------------------
# prompt emphasis grammar
# ------------------------------------------------------------------------------------------------
def split_parentheses(s: str) -> list[str]:
    """Split into top-level parenthesised groups and plain runs."""
    out, cur, depth = [], "", 0
    for ch in s:
        if ch == "(":
            if depth == 0 and cur:
                out.append(cur)
                cur = ""
            cur += ch
            depth += 1
        elif ch == ")":
            depth -= 1
            cur += ch
            if depth == 0:
                out.append(cur)
                cur = ""
        else:
            cur += ch
    if cur:
        out.append(cur)
    return out


def weighted_segments(s: str, weight: float = 1.0) -> list[tuple[str, float]]:
    """``(text)`` multiplies by 1.1, ``(text:w)`` sets w; nests recursively."""
    res = []
    for part in split_parentheses(s):
        if len(part) >= 2 and part[0] == "(" and part[-1] == ")":
            inner = part[1:-1]
            w = weight * 1.1
            c = inner.rfind(":")
            if c > 0:
                try:
                    w = float(inner[c + 1:])
                    inner = inner[:c]
                except ValueError:
                    pass
            res.extend(weighted_segments(inner, w))
        else:
            res.append((part, weight))
    return res


_ESC = (("\\)", "\0\1"), ("\\(", "\0\2"))


def escape_important(t: str) -> str:
    for a, b in _ESC:
        t = t.replace(a, b)
    return t


def unescape_important(t: str) -> str:
    t = t.replace("\0\1", ")")
    return t.replace("\0\2", "(")


# ------------------------------------------------------------------------------------------------
# textual inversion
# ------------------------------------------------------------------------------------------------
def load_embedding(name: str, directories, size: int, key: str | None = None):
    """Load a textual-inversion embedding (safetensors / weights-only pt) -> [n, size] or None."""
    if isinstance(directories, str):
        directories = [directories]
    directories = [d for d in (directories or []) if d]
    cand = None
    for d in directories:
        base = os.path.abspath(d)
        p = os.path.abspath(os.path.join(d, name))
        if os.path.commonpath([base, p]) != base:
            continue
        for ext in ("", ".safetensors", ".pt", ".bin"):
            if os.path.isfile(p + ext):
                cand = p + ext
                break
        if cand:
            break
    if cand is None:
        return None
    try:
        if cand.endswith(".safetensors"):
            from ..runtime.checkpoint import load_state_dict
            sd = load_state_dict(cand)
        else:
            sd = torch.load(cand, map_location="cpu", weights_only=True)
    except Exception as e:
        logging.warning("failed to load embedding %s: %s", cand, e)
        return None
    if "string_to_param" in sd:
        vals = list(sd["string_to_param"].values())
        emb = vals[0]
    elif key is not None and key in sd:
        emb = sd[key]
    elif isinstance(sd, dict) and len(sd) == 1:
        emb = next(iter(sd.values()))
    else:
        emb = None
        for v in sd.values() if isinstance(sd, dict) else []:
            if isinstance(v, torch.Tensor) and v.shape[-1] == size:
                emb = v
                break
    if emb is None or emb.shape[-1] != size:
        return None
    return emb.reshape(-1, size).float()


# ------------------------------------------------------------------------------------------------
# tokenizer
# ------------------------------------------------------------------------------------------------
class SDTokenizer:
    def __init__(self, max_length=77, pad_with_end=True, embedding_directory=None, embedding_size=768,
                 embedding_key="clip_l", has_start_token=True, pad_to_max_length=True, min_length=None):
        self.tok = get_clip_tokenizer()
        self.max_length = max_length
        self.min_length = min_length
        self.start_token = self.tok.BOS if has_start_token else None
        self.end_token = self.tok.EOS
        self.pad_with_end = pad_with_end
        self.pad_to_max_length = pad_to_max_length
        self.embedding_directory = embedding_directory
        self.embedding_size = embedding_size
        self.embedding_key = embedding_key
        self.max_word_length = 8
        self.embedding_identifier = "embedding:"

    def _embedding(self, name):
        e = load_embedding(name, self.embedding_directory, self.embedding_size, self.embedding_key)
        if e is None:
            s = name.strip(",")
            if len(s) < len(name):
                return load_embedding(s, self.embedding_directory, self.embedding_size, self.embedding_key), name[len(s):]
        return e, ""

    def tokenize_with_weights(self, text: str, return_word_ids=False):
        pad = self.end_token if self.pad_with_end else 0
        words = []
        for seg, w in weighted_segments(escape_important(text), 1.0):
            for word in unescape_important(seg).replace("\n", " ").split(" "):
                if not word:
                    continue
                if word.startswith(self.embedding_identifier) and self.embedding_directory is not None:
                    name = word[len(self.embedding_identifier):].strip("\n")
                    emb, rest = self._embedding(name)
                    if emb is None:
                        logging.warning("warning, embedding:%s does not exist, ignoring", name)
                    else:
                        words.append([(emb[i], w) for i in range(emb.shape[0])])
                    if not rest:
                        continue
                    word = rest
                words.append([(t, w) for t in self.tok.encode(word)])

        chunks = []
        cur = [] if self.start_token is None else [(self.start_token, 1.0, 0)]
        chunks.append(cur)
        limit = self.max_length - 1
        for wi, group in enumerate(words):
            large = len(group) >= self.max_word_length
            while group:
                if len(group) + len(cur) > limit:
                    room = self.max_length - len(cur) - 1
                    if large:
                        cur.extend((t, w, wi + 1) for t, w in group[:room])
                        cur.append((self.end_token, 1.0, 0))
                        group = group[room:]
                    else:
                        cur.append((self.end_token, 1.0, 0))
                        if self.pad_to_max_length:
                            cur.extend([(pad, 1.0, 0)] * room)
                    cur = [] if self.start_token is None else [(self.start_token, 1.0, 0)]
                    chunks.append(cur)
                else:
                    cur.extend((t, w, wi + 1) for t, w in group)
                    group = []
        cur.append((self.end_token, 1.0, 0))
        if self.pad_to_max_length:
            cur.extend([(pad, 1.0, 0)] * (self.max_length - len(cur)))
        if self.min_length is not None and len(cur) < self.min_length:
            cur.extend([(pad, 1.0, 0)] * (self.min_length - len(cur)))
        if not return_word_ids:
            chunks = [[(t, w) for t, w, _ in c] for c in chunks]
        return chunks

    def untokenize(self, pairs):
        return [(p, self.tok.decoder.get(p[0], "")) for p in pairs]


# ------------------------------------------------------------------------------------------------
# encoder
# ------------------------------------------------------------------------------------------------
class SDClipModel(torch.nn.Module):
    """One CLIP text tower + layer-selection options (sd1_clip.py:SDClipModel)."""

    LAYERS = ("last", "pooled", "hidden")

    def __init__(self, config=CLIP_L_CONFIG, layer="last", layer_idx=None, special_tokens=None,
                 layer_norm_hidden_state=True, return_projected_pooled=True, dtype=None, device=None,
                 enable_attention_masks=False):
        super().__init__()
        self.transformer = CLIPTextModel(config, dtype=dtype, device=device)
        self.num_layers = self.transformer.num_layers
        self.special_tokens = special_tokens or {"start": 49406, "end": 49407, "pad": 49407}
        self.layer_norm_hidden_state = layer_norm_hidden_state
        self.return_projected_pooled = return_projected_pooled
        self.enable_attention_masks = enable_attention_masks
        self.options_default = (layer, layer_idx, return_projected_pooled)
        self.set_layer(layer, layer_idx)

    def set_layer(self, layer, layer_idx=None):
        assert layer in self.LAYERS
        if layer == "hidden":
            assert layer_idx is not None and abs(layer_idx) <= self.num_layers
        self.layer = layer
        self.layer_idx = layer_idx

    def set_clip_options(self, options):
        li = options.get("layer", self.layer_idx)
        self.return_projected_pooled = options.get("projected_pooled", self.return_projected_pooled)
        if li is None or abs(li) > self.num_layers:
            self.set_layer("last")
        else:
            self.set_layer("hidden", li)

    def reset_clip_options(self):
        self.set_layer(self.options_default[0], self.options_default[1])
        self.return_projected_pooled = self.options_default[2]

    def _device_dtype(self):
        w = self.transformer.text_model.embeddings.token_embedding.weight
        return w.device, w.dtype

    def encode(self, token_lists):
        """token_lists: list of lists of (int | tensor) -> (z [n,77,C] fp32, pooled [n,P] fp32)."""
        device, dtype = self._device_dtype()
        emb_table = self.transformer.text_model.embeddings.token_embedding.weight
        ids = torch.tensor([[t if isinstance(t, int) else 0 for t in row] for row in token_lists],
                           dtype=torch.long)
        embeds = None
        if any(not isinstance(t, int) for row in token_lists for t in row):
            embeds = emb_table[ids.to(device)].clone()
            for r, row in enumerate(token_lists):
                for c, t in enumerate(row):
                    if not isinstance(t, int):
                        embeds[r, c] = t.to(device=device, dtype=embeds.dtype)
            # argmax pooling must still find the end token
        ids_dev = ids.to(device)
        inter_idx = self.layer_idx if self.layer == "hidden" else None
        x, inter, proj, pooled = self.transformer(ids_dev, embeds=embeds, intermediate_output=inter_idx,
                                                  final_layer_norm_intermediate=self.layer_norm_hidden_state)
        z = x if self.layer == "last" else inter
        if self.layer == "pooled":
            z = pooled[:, None, :]
        p = proj if self.return_projected_pooled else pooled
        return z.float(), p.float()

    def gen_empty_tokens(self, length):
        st = self.special_tokens
        out = []
        if st.get("start") is not None:
            out.append(st["start"])
        if st.get("end") is not None:
            out.append(st["end"])
        out += [st.get("pad", st.get("end"))] * (length - len(out))
        return out

    def encode_token_weights(self, pairs):
        """pairs: list of 77-long chunks of (token, weight) -> (z [1, 77k, C], pooled [1, P])."""
        sections = len(pairs)
        rows = [[t for t, _ in chunk] for chunk in pairs]
        maxlen = max((len(r) for r in rows), default=77)
        has_w = any(w != 1.0 for chunk in pairs for _, w in chunk)
        if has_w or sections == 0:
            rows.append(self.gen_empty_tokens(maxlen))
        out, pooled = self.encode(rows)
        # conditioning stays where node outputs live (the device: dm.intermediate_device) -- no
        # D2H + H2D round trip per prompt encode before sampling
        dev = dm.intermediate_device()
        first_pooled = pooled[0:1].to(dev)
        if sections == 0:
            return out[-1:].to(dev), first_pooled
        z = out[:sections]
        if has_w:
            wt = torch.tensor([[w for _, w in chunk] for chunk in pairs], dtype=z.dtype, device=z.device)
            z_empty = out[-1:]
            z = (z - z_empty) * wt[..., None] + z_empty
        return z.reshape(1, -1, z.shape[-1]).to(dev), first_pooled

    def load_sd(self, sd):
        return self.transformer.load_state_dict(sd, strict=False)


# ------------------------------------------------------------------------------------------------
# family stacks
# ------------------------------------------------------------------------------------------------
class _Stack(torch.nn.Module):
    """Holds named towers ``clip_l`` / ``clip_g`` / ``clip_h``; keys ``clip_x.transformer.*``."""
    tokenizer_specs = {}

    def __init__(self):
        super().__init__()

    def tokenizers(self, embedding_directory=None):
        return {n: SDTokenizer(embedding_directory=embedding_directory, **spec) for n, spec in self.tokenizer_specs.items()}

    def set_clip_options(self, options):
        for n in self.tokenizer_specs:
            getattr(self, "clip_" + n).set_clip_options(options)

    def reset_clip_options(self):
        for n in self.tokenizer_specs:
            getattr(self, "clip_" + n).reset_clip_options()

    def load_sd(self, sd):
        """Dispatch a converted state dict by prefix (clip_l./clip_g./clip_h.)."""
        missing, unexpected = [], []
        for n in self.tokenizer_specs:
            pre = f"clip_{n}."
            sub = {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}
            if sub:
                m, u = getattr(self, "clip_" + n).transformer.load_state_dict(
                    {k[len("transformer."):]: v for k, v in sub.items() if k.startswith("transformer.")}, strict=False)
                missing += [pre + x for x in m]
                unexpected += [pre + x for x in u]
        return missing, unexpected


class SD1ClipModel(_Stack):
    tokenizer_specs = {"l": dict(embedding_size=768, embedding_key="clip_l")}

    def __init__(self, dtype=None, device=None):
        super().__init__()
        self.clip_l = SDClipModel(CLIP_L_CONFIG, layer="last", dtype=dtype, device=device)

    def encode_token_weights(self, tw):
        return self.clip_l.encode_token_weights(tw["l"])


class SD2ClipModel(_Stack):
    tokenizer_specs = {"h": dict(pad_with_end=False, embedding_size=1024, embedding_key="clip_h")}

    def __init__(self, dtype=None, device=None):
        super().__init__()
        self.clip_h = SDClipModel(CLIP_H_CONFIG, layer="hidden", layer_idx=-2,
                                  special_tokens={"start": 49406, "end": 49407, "pad": 0}, dtype=dtype, device=device)

    def encode_token_weights(self, tw):
        return self.clip_h.encode_token_weights(tw["h"])


class SDXLClipModel(_Stack):
    tokenizer_specs = {"l": dict(embedding_size=768, embedding_key="clip_l"),
                       "g": dict(pad_with_end=False, embedding_size=1280, embedding_key="clip_g")}

    def __init__(self, dtype=None, device=None):
        super().__init__()
        self.clip_l = SDClipModel(CLIP_L_CONFIG, layer="hidden", layer_idx=-2, layer_norm_hidden_state=False,
                                  dtype=dtype, device=device)
        self.clip_g = SDClipModel(CLIP_G_CONFIG, layer="hidden", layer_idx=-2, layer_norm_hidden_state=False,
                                  special_tokens={"start": 49406, "end": 49407, "pad": 0}, dtype=dtype, device=device)

    def encode_token_weights(self, tw):
        g_out, g_pooled = self.clip_g.encode_token_weights(tw["g"])
        l_out, _ = self.clip_l.encode_token_weights(tw["l"])
        n = min(g_out.shape[1], l_out.shape[1])
        return torch.cat([l_out[:, :n], g_out[:, :n]], dim=-1), g_pooled


class SDXLRefinerClipModel(_Stack):
    tokenizer_specs = {"g": dict(pad_with_end=False, embedding_size=1280, embedding_key="clip_g")}

    def __init__(self, dtype=None, device=None):
        super().__init__()
        self.clip_g = SDClipModel(CLIP_G_CONFIG, layer="hidden", layer_idx=-2, layer_norm_hidden_state=False,
                                  special_tokens={"start": 49406, "end": 49407, "pad": 0}, dtype=dtype, device=device)

    def encode_token_weights(self, tw):
        return self.clip_g.encode_token_weights(tw["g"])


class StableCascadeClipModel(_Stack):
    tokenizer_specs = {"g": dict(pad_with_end=True, embedding_size=1280, embedding_key="clip_g")}

    def __init__(self, dtype=None, device=None):
        super().__init__()
        self.clip_g = SDClipModel(CLIP_G_CONFIG, layer="hidden", layer_idx=-1, layer_norm_hidden_state=False,
                                  special_tokens={"start": 49406, "end": 49407, "pad": 49407},
                                  enable_attention_masks=True, dtype=dtype, device=device)

    def encode_token_weights(self, tw):
        return self.clip_g.encode_token_weights(tw["g"])


class ClipStackTokenizer:
    def __init__(self, stack_cls, embedding_directory=None):
        self.parts = {n: SDTokenizer(embedding_directory=embedding_directory, **spec)
                      for n, spec in stack_cls.tokenizer_specs.items()}

    def tokenize_with_weights(self, text, return_word_ids=False):
        return {n: t.tokenize_with_weights(text, return_word_ids) for n, t in self.parts.items()}

    def untokenize(self, pairs):
        return next(iter(self.parts.values())).untokenize(pairs)
