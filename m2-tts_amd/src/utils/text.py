"""Text frontend: normalisation, rule/lexicon G2P, phoneme ids.

Drop-in for the reference ``src/utils/text.py`` (same public names and
outputs; pinned by tests/golden/text_ids.json, generated from the reference).
Pure Python; it feeds ``phoneme_ids`` to the GPU path and does no arithmetic
on it.  Reference behaviours kept on purpose:
  * abbreviations are expanded by plain substring replacement in a fixed
    order, so e.g. "first." becomes "firsaint" (text.py:30-49);
  * only whole tokens "0".."20" are spelled out (text.py:52-81);
  * ``length`` counts the non-SIL phonemes, while position 0 is the leading
    SIL - the text encoder therefore masks the last real phonemes and the
    final SIL (text.py:346), reproduced as-is.
"""
from __future__ import annotations

import logging
import re
import string
import unicodedata
from pathlib import Path
from typing import Dict, List, Optional

logger = logging.getLogger(__name__)

# 15 vowels, 24 consonants, then SIL / SP / UNK: ids 0..41 (reference text.py:14-23).
PHONEME_SET = ("AA AE AH AO AW AY EH ER EY IH IY OW OY UH UW "
               "B CH D DH F G HH JH K L M N NG P R S SH T TH V W Y Z ZH "
               "SIL SP UNK").split()
PHONEME_TO_ID = {p: i for i, p in enumerate(PHONEME_SET)}
ID_TO_PHONEME = dict(enumerate(PHONEME_SET))

# Applied in this order, as substring replacements on the lower-cased text.
_ABBREVIATIONS = (("dr.", "doctor"), ("mr.", "mister"), ("mrs.", "missus"), ("ms.", "miss"),
                  ("st.", "saint"), ("etc.", "et cetera"), ("vs.", "versus"), ("e.g.", "for example"),
                  ("i.e.", "that is"), ("&", "and"))

_NUMBER_WORDS = ("zero one two three four five six seven eight nine ten eleven twelve thirteen "
                 "fourteen fifteen sixteen seventeen eighteen nineteen twenty").split()
_NUMBERS = {str(i): w for i, w in enumerate(_NUMBER_WORDS)}

# The reference's small pronunciation lexicon (word -> ARPAbet).
_LEXICON_SRC = """
hello HH EH L OW|world W ER L D|the DH AH|and AE N D|to T UW|a AH|of AH V|in IH N|is IH Z|it IH T
you Y UW|that DH AE T|he HH IY|was W AH Z|for F ER|on AO N|are AA R|as AE Z|with W IH TH|his HH IH Z
they DH EY|i AY|at AE T|be B IY|this DH IH S|have HH AE V|from F R AH M|or ER|one W AH N|had HH AE D
by B AY|word W ER D|but B AH T|not N AA T|what W AH T|all AO L|were W ER|we W IY|when W EH N|your Y ER
can K AE N|said S EH D|there DH EH R|each IY CH|which W IH CH|do D UW|how HH AW|their DH EH R|if IH F
will W IH L|up AH P|other AH DH ER|about AH B AW T|out AW T|many M EH N IY|then DH EH N|them DH EH M
these DH IY Z|so S OW|some S AH M|her HH ER|would W UH D|make M EY K|like L AY K|into IH N T UW|him HH IH M
time T AY M|two T UW|more M ER|go G OW|no N OW|way W EY|could K UH D|my M AY|than DH AE N|first F ER S T
been B IH N|call K AO L|who HH UW|its IH T S|now N AW|find F AY N D|long L AO NG|down D AW N|day D EY
did D IH D|get G EH T|come K AH M|made M EY D|may M EY|part P AA R T
"""
_LEXICON = {}
for _entry in _LEXICON_SRC.replace("\n", "|").split("|"):
    _toks = _entry.split()
    if _toks:
        _LEXICON[_toks[0]] = _toks[1:]

# Letter-to-sound fallback (reference text.py:216-243): one phoneme per known letter.
_LETTER_SOUNDS = dict(zip("bcdfghjklmnpqrstvwxyz",
                          "B K D F G HH JH K L M N P K R S T V W K Y Z".split()))
_LETTER_SOUNDS.update({"a": "AE", "e": "EH", "i": "IH", "o": "AO", "u": "UH"})


def expand_abbreviations(text: str) -> str:
    out = text.lower()
    for abbr, full in _ABBREVIATIONS:
        out = out.replace(abbr, full)
    return out


def expand_numbers(text: str) -> str:
    words = []
    for word in text.split():
        core = word.strip(string.punctuation)
        if core.isdigit() and core in _NUMBERS:
            lead = word[: len(word) - len(word.lstrip(string.punctuation))]
            trail = word[len(word.rstrip(string.punctuation)):]
            word = lead + _NUMBERS[core] + trail
        words.append(word)
    return " ".join(words)


def normalize_text(text: str) -> str:
    text = unicodedata.normalize("NFD", text.lower())
    text = expand_numbers(expand_abbreviations(text))
    return re.sub(r"\s+", " ", text.strip())


class SimpleG2P:
    """Lexicon lookup with a letter-to-sound fallback; SP between words, SIL
    at both ends (reference text.py:104-282)."""

    def __init__(self):
        self.word_to_phonemes: Dict[str, List[str]] = {w: list(p) for w, p in _LEXICON.items()}

    def _grapheme_to_phoneme_fallback(self, word: str) -> List[str]:
        phones = [_LETTER_SOUNDS[ch] for ch in word.lower() if ch in _LETTER_SOUNDS]
        return phones or ["UNK"]

    def convert(self, text: str) -> List[str]:
        phones: List[str] = []
        for word in normalize_text(text).split():
            core = word.strip(string.punctuation)
            phones.extend(self.word_to_phonemes.get(core) or self._grapheme_to_phoneme_fallback(core))
            phones.append("SP")
        if phones and phones[-1] == "SP":
            phones.pop()
        return ["SIL"] + phones + ["SIL"]


class TextProcessor:
    """text -> phonemes -> ids, with optional SIL padding / truncation
    (reference text.py:285-347)."""

    def __init__(self, vocab_size: int = 256):
        self.vocab_size = vocab_size
        self.g2p = SimpleG2P()
        self.phoneme_to_id = PHONEME_TO_ID
        self.id_to_phoneme = ID_TO_PHONEME
        logger.info(f"TextProcessor initialized with {len(PHONEME_SET)} phonemes")

    def text_to_phonemes(self, text: str) -> List[str]:
        return self.g2p.convert(text)

    def phonemes_to_ids(self, phonemes: List[str]) -> List[int]:
        unk = self.phoneme_to_id["UNK"]
        return [self.phoneme_to_id.get(p, unk) for p in phonemes]

    def ids_to_phonemes(self, ids: List[int]) -> List[str]:
        return [self.id_to_phoneme.get(i, "UNK") for i in ids]

    def process_text(self, text: str, max_length: Optional[int] = None) -> Dict:
        phonemes = self.text_to_phonemes(text)
        ids = self.phonemes_to_ids(phonemes)
        if max_length is not None:
            if len(ids) > max_length:
                ids, phonemes = ids[:max_length], phonemes[:max_length]
            else:
                pad = max_length - len(ids)
                ids = ids + [self.phoneme_to_id["SIL"]] * pad
                phonemes = phonemes + ["SIL"] * pad
        return {"text": text, "phonemes": phonemes, "phoneme_ids": ids,
                "length": sum(1 for p in phonemes if p != "SIL")}


def create_phoneme_dict_file(output_path: Path) -> None:
    with open(output_path, "w") as f:
        for i, p in enumerate(PHONEME_SET):
            f.write(f"{p}\t{i}\n")
    logger.info(f"Created phoneme dictionary at {output_path}")
