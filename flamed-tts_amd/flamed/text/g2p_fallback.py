"""Offline grapheme-to-phoneme fallback.  The reference uses a LibriSpeech lexicon (missing from the
snapshot) plus g2p_en (not installable offline).  This rule-based letter/digraph mapper produces
ARPAbet tokens so the CLI runs end to end offline; it is NOT a faithful G2P and only matters for
the plumbing configuration (SURVEY.md §7 hard part 6)."""
import re

_DIGRAPHS = {"ch": ["CH"], "sh": ["SH"], "th": ["TH"], "ph": ["F"], "ng": ["NG"], "ck": ["K"], "ee": ["IY1"],
             "oo": ["UW1"], "ou": ["AW1"], "ai": ["EY1"], "ay": ["EY1"], "oa": ["OW1"], "wh": ["W"], "qu": ["K", "W"]}
_LETTERS = {"a": ["AE1"], "b": ["B"], "c": ["K"], "d": ["D"], "e": ["EH1"], "f": ["F"], "g": ["G"], "h": ["HH"],
            "i": ["IH1"], "j": ["JH"], "k": ["K"], "l": ["L"], "m": ["M"], "n": ["N"], "o": ["OW1"], "p": ["P"],
            "q": ["K"], "r": ["R"], "s": ["S"], "t": ["T"], "u": ["AH1"], "v": ["V"], "w": ["W"], "x": ["K", "S"],
            "y": ["Y"], "z": ["Z"]}


class G2pFallback:
    def __call__(self, word: str):
        w = word.lower()
        if not re.search(r"[a-z]", w):
            return [w] if w.strip() else [" "]
        out, i = [], 0
        while i < len(w):
            if w[i:i + 2] in _DIGRAPHS:
                out += _DIGRAPHS[w[i:i + 2]]
                i += 2
                continue
            out += _LETTERS.get(w[i], [])
            i += 1
        return out
