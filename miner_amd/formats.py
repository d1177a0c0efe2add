"""Data and artifact formats on either side of the scoring path.

* ``read_news_tsv`` / ``read_behaviors_tsv``: MIND news.tsv / behaviors.tsv (column map of
  src/constants.py:1-10) into the news-id layout the gather kernel consumes — the semantics of the
  reference's eval reader (src/reader.py:41-56, :89-130, :355-379):
    - impression id = the behaviors line index (lines that are dropped still use up their id);
    - the history keeps the OLDEST ``his_length`` clicks, left-padded with the pad news (:368-369);
    - an impression is kept only if its behavior column contains both a "-1" and a "-0" (:374);
    - his_mask = clicked news' category != the pad category (src/entities.py:395), categories
      mapped with ``category2id.get(c, category2id['unk'])`` (:115);
  table rows: 0 = the pad news, 1 + i = line i of news.tsv.
* ``load_news_table``: the news encoder's output for every news item (row layout above) from
  .npy / .safetensors / a weights-only torch file — loaders that execute nothing from the file.
* ``save_predictions``: preds.pkl exactly as SlowEvaluator writes it (src/evaluation.py:173-175):
  {'pred': [[p] per eval sample], 'impression_id': [id per sample]}, samples impression-major.
* ``load_miner_state_dict``: reference checkpoints are pickled whole modules
  (src/base_trainer.py:204-235) and are not unpickled here; export ``model.state_dict()`` in the
  reference environment and load it with ``torch.load(weights_only=True)``: the parameter names of
  miner_amd.model match the reference's.
"""
from __future__ import annotations

import csv
import dataclasses
import json
import os
import pickle
from typing import Dict, List, Optional

import numpy as np
import torch

from .synthetic import Behaviors

# src/constants.py:1-10
USER_ID, HISTORY, BEHAVIOR = 1, 3, 4
NEWS_ID, TITLE, CATEGORY, SAPO = 0, 1, 2, 3


@dataclasses.dataclass
class NewsIndex:
    row: Dict[str, int]          # news id -> table row (0 = pad)
    category: np.ndarray         # [n_rows] int64 category id per row (row 0: category2id['pad'])
    titles: List[str]            # per row ('' for the pad row), for an external news encoder
    pad_category: int

    @property
    def n_rows(self) -> int:
        return len(self.titles)


def read_category2id(path: str) -> Dict[str, int]:
    with open(path, encoding="utf-8") as f:
        return json.load(f)


def read_news_tsv(path: str, category2id: Dict[str, int]) -> NewsIndex:
    rows, cats, titles = {}, [category2id["pad"]], [""]
    with open(path, mode="r", encoding="utf-8", newline="") as f:
        for line in csv.reader(f, delimiter="\t"):
            rows[line[NEWS_ID]] = len(titles)
            cats.append(category2id.get(line[CATEGORY], category2id["unk"]))
            titles.append(line[TITLE])
    return NewsIndex(rows, np.asarray(cats, np.int64), titles, category2id["pad"])


def read_behaviors_tsv(path: str, news: NewsIndex, his_length: int, device="cpu") -> Behaviors:
    """behaviors.tsv -> Behaviors (batched layout: one row of candidates per kept impression)."""
    his, cand, lab, sizes, ids = [], [], [], [], []
    with open(path, mode="r", encoding="utf-8", newline="") as f:
        for i, line in enumerate(csv.reader(f, delimiter="\t")):
            beh = line[BEHAVIOR]
            if not ("-1" in beh and "-0" in beh):            # reader.py:374
                continue
            clicked = [news.row[n] for n in line[HISTORY].split()]   # KeyError on unknown news, as the reference
            clicked = [0] * (his_length - len(clicked)) + clicked[:his_length]
            his.append(clicked)
            n = 0
            for b in beh.split():
                nid, label = b.split("-")
                cand.append(news.row[nid])
                lab.append(int(label))
                n += 1
            sizes.append(n)
            ids.append(i)
    his_rows = np.asarray(his, np.int64).reshape(-1, his_length)
    mask = news.category[his_rows] != news.pad_category
    offs = np.zeros(len(sizes) + 1, np.int64)
    offs[1:] = np.cumsum(sizes)
    dev = torch.device(device)
    return Behaviors(torch.from_numpy(his_rows).to(dev, torch.int32), torch.from_numpy(mask).to(dev),
                     torch.as_tensor(cand, dtype=torch.int32).to(dev), torch.from_numpy(offs).to(dev, torch.int32),
                     torch.as_tensor(lab, dtype=torch.uint8).to(dev), torch.as_tensor(ids, dtype=torch.int64).to(dev))


def load_news_table(path: str, key: Optional[str] = None) -> torch.Tensor:
    """[n_rows, d] news embeddings (row 0 = pad news) from .npy, .safetensors or a torch file
    holding a tensor or a dict of tensors (weights_only)."""
    if path.endswith(".npy"):
        return torch.from_numpy(np.load(path, allow_pickle=False))
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        t = load_file(path)
        return t[key] if key else next(iter(t.values()))
    obj = torch.load(path, map_location="cpu", weights_only=True)
    return obj[key] if isinstance(obj, dict) else obj


def save_predictions(path: str, probs: torch.Tensor, impression_ids: torch.Tensor,
                     cand_offsets: Optional[torch.Tensor] = None) -> str:
    """preds.pkl of SlowEvaluator.save_predictions (evaluation.py:173-175) from batched scores:
    one [p] entry per eval sample, impression-major, with the sample's impression id."""
    p = probs.detach().float().cpu().reshape(-1)
    if cand_offsets is None:
        sizes = np.full(impression_ids.numel(), p.numel() // max(impression_ids.numel(), 1))
    else:
        sizes = np.diff(cand_offsets.cpu().numpy().astype(np.int64))
    ids = np.repeat(impression_ids.cpu().numpy().astype(np.int64), sizes)
    out = os.path.join(path, "preds.pkl")
    with open(out, "wb") as f:
        if ids.size and (ids.min() < 0 or ids.max() >= 2 ** 31):
            pickle.dump({"pred": [[float(x)] for x in p.tolist()], "impression_id": ids.tolist()}, f)
        else:
            f.write(preds_pickle(p.numpy(), ids))
    return out


def preds_pickle(probs: np.ndarray, ids: np.ndarray) -> bytes:
    """The pickle stream of {"pred": [[p], ...], "impression_id": [id, ...]} (protocol 2), written
    with numpy instead of building 2·N Python objects: pickle.load returns exactly the structure
    SlowEvaluator.save_predictions pickles (evaluation.py:173-175; floats are the fp32 probabilities
    widened to double, as float() does). ids must lie in [0, 2^31)."""
    n = probs.size
    items = np.empty((n, 11), np.uint8)               # ']' 'G' <8-byte big-endian double> 'a'
    items[:, 0] = ord("]")
    items[:, 1] = ord("G")
    items[:, 2:10] = probs.astype(">f8").view(np.uint8).reshape(n, 8)
    items[:, 10] = ord("a")
    ints = np.empty((ids.size, 5), np.uint8)          # 'J' <4-byte little-endian int>
    ints[:, 0] = ord("J")
    ints[:, 1:] = ids.astype("<i4").view(np.uint8).reshape(ids.size, 4)

    def key(k: str) -> bytes:
        b = k.encode()
        return b"X" + len(b).to_bytes(4, "little") + b

    return b"".join([b"\x80\x02}(", key("pred"), b"](", items.tobytes(), b"e", key("impression_id"), b"](",
                     ints.tobytes(), b"eu."])


def load_miner_state_dict(model: torch.nn.Module, path: str, strict: bool = False):
    """Load a reference Miner state_dict (exported with torch.save(model.state_dict())) into a
    miner_amd.model.Miner. News-encoder keys load when the model has that encoder; with
    strict=False the scoring parameters alone are enough."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    return model.load_state_dict(sd, strict=strict)
