"""Generate tests/golden/reader_mind.npz (+ the tsv inputs under tests/golden/mind_tiny/) by running
the REFERENCE's own eval reader (src/reader.py:41-56 read_eval_dataset, :355-379
_parse_eval_line, :89-130 _read_news_info) on a tiny hand-made MIND-format dataset.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_reader_golden.py

The reference tokenizer (RoBERTa) is not available offline; a stub tokenizer stands in (the
reader only needs cls/eos/pad ids and encode(); token ids do not enter the recorded arrays). What
is recorded, per eval sample in the reference's order: impression id, the clicked-news ids
(news-id strings, mapped to table rows = 1 + line index of news.tsv, 0 = the pad news), the
candidate news row, the label and his_mask (entities.py:395: category != pad). Data only: no
reference code is stored.
"""
from __future__ import annotations

import csv
import json
import os
import sys

import numpy as np

REF = os.environ.get("MINER_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
TINY = os.path.join(HERE, "mind_tiny")
HIS_LENGTH = 6

NEWS = [  # news_id, title, category, sapo
    ("N1", "a", "sports", "x"), ("N2", "b", "news", "y"), ("N3", "c", "finance", "z"),
    ("N4", "d", "sports", "w"), ("N5", "e", "weather", "v"), ("N6", "f", "unseen_cat", "u"),
    ("N7", "g", "news", "t"), ("N8", "h", "sports", "s"), ("N9", "i", "finance", "r"),
    ("N10", "j", "news", "q"), ("N11", "k", "autos", "p"), ("N12", "l", "sports", "o"),
]
BEHAVIORS = [  # impression id, user, time, history, behaviors
    ("1", "U1", "t", "N1 N2 N3", "N4-1 N5-0 N6-0"),
    ("2", "U2", "t", "", "N7-0 N8-1"),                                     # empty history
    ("3", "U3", "t", "N1 N2 N3 N4 N5 N6 N7 N8 N9", "N10-1 N11-0"),         # history > his_length
    ("4", "U1", "t", "N5", "N1-1 N2-1"),                                   # no non-click: dropped
    ("5", "U4", "t", "N2 N9", "N3-0 N4-0"),                                # no click: dropped
    ("6", "U9", "t", "N6 N11", "N12-0 N9-1 N1-0 N2-1"),                   # unknown user; 'unseen_cat'
    ("7", "U2", "t", "N3 N3 N3 N3 N3 N3", "N5-1 N6-0"),                    # exactly his_length, repeats
]
CATEGORY2ID = {"pad": 0, "unk": 1, "sports": 2, "news": 3, "finance": 4, "weather": 5, "autos": 6}
USER2ID = {"pad": 0, "unk": 1, "U1": 2, "U2": 3, "U3": 4, "U4": 5}


class StubTokenizer:
    cls_token_id, eos_token_id, pad_token_id = 0, 2, 1

    def encode(self, text, add_special_tokens=True, truncation=True, max_length=None):
        ids = [self.cls_token_id] + [3 + (ord(ch) % 50) for ch in text] + [self.eos_token_id]
        return ids[:max_length] if max_length else ids


def write_inputs():
    os.makedirs(TINY, exist_ok=True)
    with open(os.path.join(TINY, "news.tsv"), "w", newline="") as f:
        w = csv.writer(f, delimiter="\t")
        for row in NEWS:
            w.writerow(row)
    with open(os.path.join(TINY, "behaviors.tsv"), "w", newline="") as f:
        w = csv.writer(f, delimiter="\t")
        for row in BEHAVIORS:
            w.writerow(row)
    with open(os.path.join(TINY, "category2id.json"), "w") as f:
        json.dump(CATEGORY2ID, f)
    with open(os.path.join(TINY, "user2id.json"), "w") as f:
        json.dump(USER2ID, f)


def main():
    write_inputs()
    if not os.path.isdir(os.path.join(REF, "src")):
        print(f"reference not found at {REF}: wrote the tsv inputs only")
        return 0
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from src.reader import Reader                          # noqa: E402  (reference)

    reader = Reader(tokenizer=StubTokenizer(), max_title_length=32, max_sapo_length=64, user2id=USER2ID,
                    category2id=CATEGORY2ID, max_his_click=HIS_LENGTH, npratio=None)
    # read_eval_dataset does not hand back the news map: run its two steps (reader.py:41-56)
    dataset, news_dataset = reader._read("tiny", os.path.join(TINY, "news.tsv"))
    with open(os.path.join(TINY, "behaviors.tsv"), newline="") as f:
        for i, line in enumerate(csv.reader(f, delimiter="\t")):
            reader._parse_eval_line(i, line, news_dataset, dataset)
    vanilla = news_dataset["vanilla"]
    row_of = {id(vanilla["pad"]): 0}
    for i, (nid, *_rest) in enumerate(NEWS):
        row_of[id(vanilla[nid])] = i + 1
    imp, his, cand, lab, mask = [], [], [], [], []
    for s in dataset.samples:
        imp.append(s.impression.impression_id)
        his.append([row_of[id(n)] for n in s.clicked_news])
        mask.append([n.category != CATEGORY2ID["pad"] for n in s.clicked_news])
        assert len(s.impression.news) == 1
        cand.append(row_of[id(s.impression.news[0])])
        lab.append(s.impression.label[0])
    path = os.path.join(HERE, "reader_mind.npz")
    np.savez_compressed(path, impression_id=np.array(imp, np.int64), his_rows=np.array(his, np.int64),
                        cand_row=np.array(cand, np.int64), label=np.array(lab, np.int64),
                        his_mask=np.array(mask, bool), his_length=np.int64(HIS_LENGTH))
    print(f"{path}: {len(imp)} eval samples from {len(BEHAVIORS)} behaviors lines")
    return 0


if __name__ == "__main__":
    sys.exit(main())
