"""TEST INFRASTRUCTURE ONLY -- CPU restatements of the reference's n-gram level helpers, used by tests/ as the
checker for protgram_directgcn_amd.ngram (never imported by the product).

* next_node_labels_ref: ProtGramDirectGCNTrainer._generate_next_node_labels
  (src/pipeline/protgram_directgcn_trainer.py:222-236): per node, the successors of A_out_w's row with the
  maximum weight; the node itself when the row is empty. The reference draws one of the tied successors with
  random.choice; this returns the whole tie set so the test can check membership.
* pool_features_ref: the level-n feature initialisation (trainer :317-330): for every n-gram, np.mean over the
  float32 embeddings of its prefix [:-1] and suffix [1:] that exist in the level-(n-1) map; zeros when neither.
* aggregate_parts_ref: data_builder.py:263-270 -- read 'source target' lines (bad lines skipped) and
  groupby(['source', 'target']).size().
"""
from typing import Dict, List, Sequence

import numpy as np
import pandas as pd


def next_node_labels_ref(num_nodes: int, src: np.ndarray, dst: np.ndarray, w: np.ndarray) -> List[set]:
    out: List[set] = []
    for i in range(num_nodes):
        m = src == i
        if not m.any():
            out.append({i})
            continue
        succ, ww = dst[m], w[m]
        out.append(set(succ[ww == ww.max()].tolist()))
    return out


def pool_features_ref(cur_strings: Sequence[str], prev_strings: Sequence[str], emb_prev: np.ndarray) -> np.ndarray:
    prev_map: Dict[str, int] = {s: i for i, s in enumerate(prev_strings)}
    x = np.zeros((len(cur_strings), emb_prev.shape[1]), dtype=np.float32)
    for idx, s in enumerate(cur_strings):
        p_idx, s_idx = prev_map.get(s[:-1]), prev_map.get(s[1:])
        pool = [emb_prev[i] for i in [p_idx, s_idx] if i is not None]
        if pool:
            x[idx] = np.mean(np.array(pool, dtype=np.float32), axis=0)
    return x


def aggregate_parts_ref(paths: Sequence[str]) -> pd.DataFrame:
    frames = [pd.read_csv(p, sep=" ", header=None, names=["source", "target"], on_bad_lines="skip") for p in paths]
    df = pd.concat(frames, ignore_index=True)
    df = df[pd.to_numeric(df["source"], errors="coerce").notna() & pd.to_numeric(df["target"], errors="coerce").notna()]
    df = df.astype({"source": np.int64, "target": np.int64})
    return df.groupby(["source", "target"]).size().to_frame(name="weight").reset_index()
