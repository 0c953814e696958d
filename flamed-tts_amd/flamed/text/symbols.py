"""Phoneme / character symbol table (reference flamed/text/symbols.py).  The ordered list is data:
symbols.json holds the reference's table (pad, special, punctuation, letters, "@"+ARPAbet, "@"+pinyin,
silences) so phoneme ids match released checkpoints."""
import json
import os

with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "symbols.json")) as _f:
    symbols = json.load(_f)
