"""Text -> symbol ids (reference flamed/text/__init__.py): plain text goes through the cleaners and
character symbols; text inside {curly braces} is ARPAbet mapped to "@"-prefixed phoneme symbols.

Adapted from https://github.com/keithito/tacotron (MIT license), as the reference's text package notes: the
`text_to_sequence` / `sequence_to_text` behaviour is kept so the symbol ids are bit-exact."""
import re

from flamed.text import cleaners
from flamed.text.symbols import symbols

_symbol_to_id = {s: i for i, s in enumerate(symbols)}
_id_to_symbol = {i: s for i, s in enumerate(symbols)}
_curly_re = re.compile(r"(.*?)\{(.+?)\}(.*)")


def _clean_text(text, cleaner_names):
    for name in cleaner_names:
        fn = getattr(cleaners, name, None)
        if fn is None:
            raise Exception("Unknown cleaner: %s" % name)
        text = fn(text)
    return text


def _should_keep_symbol(s):
    return s in _symbol_to_id and s != "_" and s != "~"


def _symbols_to_sequence(syms):
    return [_symbol_to_id[s] for s in syms if _should_keep_symbol(s)]


def _arpabet_to_sequence(text):
    return _symbols_to_sequence(["@" + s for s in text.split()])


def text_to_sequence(text, cleaner_names):
    seq = []
    while len(text):
        m = _curly_re.match(text)
        if not m:
            seq += _symbols_to_sequence(_clean_text(text, cleaner_names))
            break
        seq += _symbols_to_sequence(_clean_text(m.group(1), cleaner_names))
        seq += _arpabet_to_sequence(m.group(2))
        text = m.group(3)
    return seq


def sequence_to_text(sequence):
    out = ""
    for sid in sequence:
        if sid in _id_to_symbol:
            s = _id_to_symbol[sid]
            if len(s) > 1 and s[0] == "@":
                s = "{%s}" % s[1:]
            out += s
    return out.replace("}{", " ")
