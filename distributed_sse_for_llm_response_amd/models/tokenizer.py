"""Tokenizers for the streaming engine.

The reference serves Mistral-7B-Instruct-v0.3 with its SentencePiece tokenizer inside vLLM
(reference ``kubernetes/base/llm/deployment.yaml:86-97``).  No tokenizer files are reachable here,
so the default is a deterministic synthetic tokenizer with the same vocabulary size (32768): every
id maps to a printable, valid-UTF-8 piece (so streamed deltas are well-formed JSON strings) and
``encode`` maps words to ids by a stable hash.  When a local HF tokenizer directory is given,
:class:`HFTokenizer` wraps it instead (``local_files_only``: nothing is downloaded).
"""
from __future__ import annotations

import json
import re
import zlib

SPECIAL = {0: "<unk>", 1: "<s>", 2: "</s>"}
_ONSETS = ["", "b", "c", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t", "v", "w", "z", "st",
           "tr", "pl", "gr", "ch", "sh", "th", "br", "cl", "fl", "sp", "qu", "dr"]
_VOWELS = ["a", "e", "i", "o", "u", "ai", "ea", "ou", "io", "y", "ie", "oo", "ei", "au", "ue", "oa"]
_CODAS = ["", "n", "r", "s", "t", "l", "m", "nd", "st", "ng", "ck", "x", "rt", "ll", "ss", "nt"]


class SyntheticTokenizer:
    """Deterministic id <-> piece mapping with a leading-space word convention (like SentencePiece)."""

    def __init__(self, vocab_size: int = 32768, bos_id: int = 1, eos_id: int = 2):
        self.vocab_size, self.bos_id, self.eos_id = vocab_size, bos_id, eos_id
        self._pieces = [self._make_piece(i) for i in range(vocab_size)]

    @staticmethod
    def _syllable(k: int) -> str:
        o = _ONSETS[k % len(_ONSETS)]
        k //= len(_ONSETS)
        v = _VOWELS[k % len(_VOWELS)]
        k //= len(_VOWELS)
        return o + v + _CODAS[k % len(_CODAS)]

    def _make_piece(self, i: int) -> str:
        if i in SPECIAL:
            return SPECIAL[i]
        if i < 3 + 10:
            return str(i - 3)
        if i < 3 + 10 + 16:
            return ".,;:!?'\"()-/&<>"[(i - 13) % 15] if (i - 13) < 15 else "\n"
        k = i - 29
        word = self._syllable(k)
        if k >= 8192:
            word += self._syllable(k // 8192 + 7)
        return (" " if i % 4 != 0 else "") + word

    def piece(self, i: int) -> str:
        return self._pieces[i] if 0 <= i < self.vocab_size else "<unk>"

    def pieces(self) -> list:
        return list(self._pieces)

    def encode(self, text: str, add_bos: bool = True) -> list:
        ids = [self.bos_id] if add_bos else []
        for w in re.findall(r"\S+", text):
            ids.append(29 + zlib.crc32(w.encode("utf-8")) % (self.vocab_size - 29))
        return ids

    def decode(self, ids) -> str:
        return "".join(self.piece(int(i)) for i in ids if int(i) not in SPECIAL)

    def chat_prompt(self, message: str) -> list:
        """[INST] message [/INST] framing of the Mistral instruct template (synthetic ids)."""
        return self.encode("[INST] " + message + " [/INST]")

    def messages_prompt(self, messages: list) -> list:
        """Multi-turn Mistral framing: <s>[INST] u1 [/INST] a1</s>[INST] u2 [/INST] (system text joins the
        first user turn, as the v0.3 template folds it into a user message)."""
        ids = [self.bos_id]
        system = " ".join(m["content"] for m in messages if m["role"] == "system")
        first = True
        for m in messages:
            if m["role"] == "user":
                text = (system + "\n\n" + m["content"]) if (first and system) else m["content"]
                ids += self.encode("[INST] " + text + " [/INST]", add_bos=False)
                first = False
            elif m["role"] == "assistant":
                ids += self.encode(m["content"], add_bos=False) + [self.eos_id]
        return ids


class HFTokenizer:
    """Local HuggingFace tokenizer directory (no network access)."""

    def __init__(self, path: str):
        from transformers import AutoTokenizer

        self.tok = AutoTokenizer.from_pretrained(path, local_files_only=True)
        self.vocab_size = len(self.tok)
        self.bos_id = self.tok.bos_token_id
        self.eos_id = self.tok.eos_token_id

    def piece(self, i: int) -> str:
        return self.tok.decode([i])

    def pieces(self) -> list:
        return [self.tok.decode([i]) for i in range(self.vocab_size)]

    def encode(self, text: str, add_bos: bool = True) -> list:
        return self.tok.encode(text, add_special_tokens=add_bos)

    def decode(self, ids) -> str:
        return self.tok.decode(list(ids), skip_special_tokens=True)

    def chat_prompt(self, message: str) -> list:
        return self.tok.apply_chat_template([{"role": "user", "content": message}], add_generation_prompt=True)

    def messages_prompt(self, messages: list) -> list:
        return self.tok.apply_chat_template(messages, add_generation_prompt=True)


def prompt_for_request(tok, req: dict) -> list:
    """Prompt ids of a queued chat request: the OpenAI `messages` conversation when the request came from
    POST /v1/chat/completions, else the single `message` of POST /chat."""
    msgs = req.get("messages")
    if msgs:
        return tok.messages_prompt(json.loads(msgs))
    return tok.chat_prompt(req["message"])


def get_tokenizer(vocab_size: int, path: str | None = None):
    return HFTokenizer(path) if path else SyntheticTokenizer(vocab_size)
