"""Ordering metrics of trainers/metrics.py: compute_metrics over predicted and
ground-truth orders, with the reference's definitions and its quirks kept:

  partial_match   mean positional accuracy (:86-94)
  exact_match     1 if the whole order matches (:95-104)
  distance_based  sum over gold items of |gold position - predicted position|; an item missing
                  from the prediction SETS the running sum to max_story_length (:105-118)
  lcs / lcs_substr  longest common subsequence / substring length (:119-132, :186-228)
  tau             1 - 2 * (#predicted ordered pairs absent from the gold order) / C(n, 2)
                  (:70-80; n = 1 divides by zero as the reference does)
  ms / wms        minimum swaps to turn the prediction into the gold order via cycle
                  decomposition; wms weights each cycle by |pos - start| of its first element
                  (:133-146, :231-296)
  head_prediction, pairwise_prediction (:158-183)

Every pair (pred, label) is first cut to the shorter length (make_same_len, :188-195). A label
list of lists is a multi-reference ground truth (:64-67): every metric tuple is computed per
reference (in METRICS order, the prediction truncated cumulatively as the reference does), the
lexicographically largest tuple is kept and averaged (:21-55, `multiref_metrics == "max"`).

Host-side Python over a few hundred small integer lists per eval; LCS is the O(mn) dynamic
program (the reference's naive recursion returns the same length).
"""
import itertools

import numpy as np

METRICS = ["partial_match", "exact_match", "lcs_substr", "lcs", "tau", "ms", "wms",
           "distance_based"]  # trainers/metrics.py:15-18


def make_same_len(pred, label):
    if not isinstance(label, list):
        label = label.tolist()
    n = min(len(pred), len(label))
    return pred[:n], label[:n]


def lcs_substr(x, y):
    """Longest common contiguous run."""
    best = 0
    prev = [0] * (len(y) + 1)
    for i in range(1, len(x) + 1):
        cur = [0] * (len(y) + 1)
        for j in range(1, len(y) + 1):
            if x[i - 1] == y[j - 1]:
                cur[j] = prev[j - 1] + 1
                best = max(best, cur[j])
        prev = cur
    return best


def lcs(x, y):
    """Longest common subsequence length."""
    prev = [0] * (len(y) + 1)
    for i in range(1, len(x) + 1):
        cur = [0] * (len(y) + 1)
        for j in range(1, len(y) + 1):
            cur[j] = prev[j - 1] + 1 if x[i - 1] == y[j - 1] else max(prev[j], cur[j - 1])
        prev = cur
    return prev[-1]


def min_swaps(pred, label, weighted=False):
    """Cycle decomposition of the map gold position -> predicted position (metrics.py:231-296):
    (cycle length - 1) per cycle, times |pred position - gold position| of the cycle's first
    element when weighted."""
    n = len(pred)
    pred = list(pred)
    target = [pred.index(x) for x in label]  # raises if a gold item is not predicted
    seen = [False] * n
    ans = 0
    for i in range(n):
        if seen[i] or target[i] == i:
            continue
        size, j = 0, i
        while not seen[j]:
            seen[j] = True
            j = target[j]
            size += 1
        if size > 0:
            ans += (size - 1) * (abs(target[i] - i) if weighted else 1)
    return ans


def _tau(p, t):
    gold = set(itertools.combinations(t, 2))
    got = set(itertools.combinations(p, 2))
    discordant = len(got) - len(got & gold)
    return 1 - 2 * discordant / (len(p) * (len(p) - 1) / 2)


def _one(args, metric, p, t):
    p, t = make_same_len(p, t)
    if metric == "tau":
        return _tau(p, t)
    if metric == "partial_match":
        return float((np.asarray(p) == np.asarray(t)).mean())
    if metric == "exact_match":
        return float(int(np.sum(np.asarray(p) == np.asarray(t))) == len(p))
    if metric == "distance_based":
        p = list(p)
        d = 0
        for j, g in enumerate(t):
            if g not in p:
                d = args.max_story_length
            else:
                d += abs(j - p.index(g))
        return d
    if metric in ("lcs", "longest_common_subsequence"):
        return lcs(p, t)
    if metric in ("lcs_substr", "longest_common_substring"):
        return lcs_substr(p, t)
    if metric == "ms":
        return min_swaps(p, t)
    if metric == "wms":
        return min_swaps(p, t, weighted=True)
    if metric == "head_prediction":
        return 1.0 if p[0] == t[0] else 0.0
    if metric == "pairwise_prediction":
        gold = {(t[j], t[k]) for j in range(len(t)) for k in range(j + 1, len(t))}
        hit = sum(1.0 for j in range(len(p)) for k in range(j + 1, len(p)) if (p[j], p[k]) in gold)
        return hit / float(len(gold))
    raise NotImplementedError(f"Metric {metric} is not implemented yet.")


def multiref_metrics(args, preds, labels):
    """Best reference per prediction by the METRICS tuple (max), averaged (metrics.py:21-55)."""
    mode = getattr(args, "multiref_metrics", None)
    if mode != "max":
        raise NotImplementedError(f"Can't deal with multiref metric: {mode} yet!")
    res = {m: 0 for m in METRICS}
    for pred, refs in zip(preds, labels):
        tuples = []
        for label in refs:
            pred, label = make_same_len(pred, label)  # the prediction stays truncated
            tuples.append(tuple(compute_metrics(args, m, [pred], [label]) for m in METRICS))
        best = max(tuples)
        for m, v in zip(METRICS, best):
            res[m] += v
    return {m: v / len(preds) for m, v in res.items()}


def compute_metrics(args, metrics, preds, labels):
    """trainers/metrics.py:58-185: mean of `metrics` over the (pred, label) pairs."""
    assert len(preds) == len(labels), (
        f"Predictions and labels have mismatched lengths {len(preds)} and {len(labels)}")
    if np.asarray(labels[0]).ndim > 1:
        return multiref_metrics(args, preds, labels)[metrics]
    acc = 0.0
    for p, t in zip(preds, labels):
        acc += _one(args, metrics, p, t)
    return acc / len(preds)
