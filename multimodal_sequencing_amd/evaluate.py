"""BERSON evaluation loop and result summary: berson_evaluate / cal_result of
models/berson/eval.py:39-368, on top of the device beam search (berson.berson_pointer_network)
and the ordering metrics (metrics.py).

Same contract as the reference: one story per batch (SequentialSampler), the gold order is
batch[3] (a [1, R, N] tensor is a multi-reference gold: its first row is used for decoding and
pmr/acc, all rows for the metrics), a one-sentence story is "predicted" as its gold order; lines
'pred|||gold' go to output_order.txt; results {'acc_dev', 'pmr_dev', 'taus_dev'} are written to
eval_results_split_{split}.txt and appended to all_eval_results.txt; with
args.eval_save_all_results a per-story all_predictions.csv (pm, em, lcs_substr, lcs, ms, wms,
dist, tau) is written.
"""
import csv
import itertools
import json
import logging
import os

import numpy as np
import torch

from .metrics import compute_metrics

logger = logging.getLogger(__name__)

_CSV_METRICS = {"pm": "partial_match", "em": "exact_match", "lcs_substr": "lcs_substr",
                "lcs": "lcs", "ms": "ms", "wms": "wms", "dist": "distance_based", "tau": "tau"}


def _flat_accuracy(truth, predicted):
    """sklearn accuracy_score over the concatenated orders (eval.py:254-255)."""
    t = list(itertools.chain.from_iterable(truth))
    p = list(itertools.chain.from_iterable(predicted))
    if len(t) != len(p):
        raise ValueError(f"Found input variables with inconsistent numbers of samples: "
                         f"[{len(t)}, {len(p)}]")
    return float(np.mean(np.asarray(t) == np.asarray(p))) if t else 0.0


def cal_result(truth, predicted, best_acc, f, args):
    """eval.py:190-368 -> (mean per-story positional accuracy, perfect-match ratio, mean tau).
    Also appends the flat accuracy to `best_acc`, closes `f`, writes the per-story performance
    csv/jsonl when args.ref_json_file is set, and logs every metric of METRICS."""
    right = total = pmr_right = 0
    taus, accs, pm_p, pm_r = [], [], [], []
    to_compare = []
    idx = 0
    multiref = False
    for t, p in zip(truth, predicted):
        t_org = t
        if np.asarray(t).ndim > 1:
            t = t[0]
            multiref = True
        if len(p) == 1:  # a one-sentence story counts as fully right
            right += 1
            total += 1
            pmr_right += 1
            accs.append(1)
            taus.append(1)
            continue
        eq = np.equal(t, p)
        right += eq.sum()
        accs.append(eq.sum() / len(t))
        total += len(t)
        pmr_right += eq.all()
        gold = set(itertools.combinations(t, 2))
        got = set(itertools.combinations(p, 2))
        pm_p.append(len(gold & got) / len(got))
        pm_r.append(len(gold & got) / len(gold))
        taus.append(1 - 2 * (len(got) - len(got & gold)) / (len(p) * (len(p) - 1) / 2))
        to_compare.append((eq.sum() / len(t), eq.all(), idx, p, t_org))
        idx += 1
    flat_truth = [t[0] for t in truth] if multiref else truth
    best_acc.append(_flat_accuracy(flat_truth, predicted))
    pmr = pmr_right / len(truth)
    taus = np.mean(taus)
    pmp, pmr_ = (np.mean(pm_p), np.mean(pm_r)) if pm_p else (0.0, 0.0)
    if pmp + pmr_ > 0:
        logger.info("pairwise-match F1: %.4f", 2 * pmp * pmr_ / (pmp + pmr_))
    if f is not None:
        f.close()
    accs = np.mean(accs)
    ref = getattr(args, "ref_json_file", None)
    if ref is not None:
        _write_performance(args, ref, to_compare)
    res = {m: compute_metrics(args, m, predicted, truth) for m in
           ["partial_match", "exact_match", "lcs", "lcs_substr", "distance_based", "ms", "wms",
            "tau"]}
    for m, v in res.items():
        logger.info("Metric: %s  Perf: %.3f", m, v)
    logger.info("& PM    & EM    & Lseq & Lstr & tau  & Dist.")
    logger.info("& {:03.2f} & {:03.2f} & {:03.2f} & {:03.2f} & {:03.2f} & {:03.2f}".format(
        res["partial_match"] * 100, res["exact_match"] * 100, res["lcs"], res["lcs_substr"],
        res["tau"], res["distance_based"]))
    return accs, pmr, taus


def _write_performance(args, ref_json_file, to_compare):
    """eval.py:283-339: per-story metrics keyed by the story url (jsonl records; RecipeQA:
    {'data': [...]} deduplicated by recipe_id) to {stem}_model_performance.csv / .jsonl."""
    recipe = "recipeQA" in ref_json_file
    with open(ref_json_file, "r") as jf:
        if recipe:
            data, used = [], set()
            for d in json.load(jf)["data"]:
                if d["recipe_id"] not in used:
                    used.add(d["recipe_id"])
                    data.append(d)
        else:
            data = [json.loads(line.strip()) for line in jf]
    stem = ref_json_file.split(".json")[0].split("/")[-1]
    mlist = ["partial_match", "exact_match", "lcs", "lcs_substr", "distance_based", "ms", "wms",
             "tau"]
    rows = []
    with open(os.path.join(args.output_dir, f"{stem}_model_performance.csv"), "w") as cf:
        w = csv.DictWriter(cf, fieldnames=["index", "url", "prediction", "gt"] + mlist)
        w.writeheader()
        for acc_c, pmr_c, i, pred, gt in to_compare:
            row = {"partial_match": acc_c, "exact_match": pmr_c, "index": i,
                   "url": data[i]["recipe_id"] if recipe else data[i]["url"],
                   "prediction": pred, "gt": gt}
            for m in mlist:
                row[m] = compute_metrics(args, m, [pred], [gt])
            w.writerow(row)
            rows.append(row)
    if recipe:
        rows = sorted(rows, key=lambda r: r["url"])
    with open(os.path.join(args.output_dir, f"{stem}_model_performance.jsonl"), "w") as of:
        for r in rows:
            of.write(json.dumps(r, default=_json_default) + "\n")


def _json_default(o):
    if isinstance(o, np.generic):
        return o.item()
    if isinstance(o, np.ndarray):
        return o.tolist()
    raise TypeError(type(o))


def berson_evaluate(args, model, load_and_cache_examples, tokenizer, prefix="",
                    data_split="test", human_evaluate=False, pointer_network=None):
    """eval.py:39-187. `load_and_cache_examples(args, [task], tokenizer, evaluate=True,
    data_split=...)` returns a map-style dataset of tuples (input_ids, attention_mask,
    token_type_ids, labels, guid, ..., images); `pointer_network` defaults to the device beam
    search berson.berson_pointer_network."""
    if pointer_network is None:
        from .berson import berson_pointer_network as pointer_network
    from torch.utils.data import DataLoader, SequentialSampler
    results = {}
    tasks = args.task_names
    for task, out_dir in zip(tasks, [args.output_dir] * len(tasks)):
        dataset = load_and_cache_examples(args, [task], tokenizer, evaluate=True,
                                          data_split=data_split)
        if not os.path.exists(out_dir) and getattr(args, "local_rank", -1) in (-1, 0):
            os.makedirs(out_dir)
        args.eval_batch_size = args.per_gpu_eval_batch_size * max(1, getattr(args, "n_gpu", 1))
        loader = DataLoader(dataset, sampler=SequentialSampler(dataset),
                            batch_size=args.eval_batch_size)
        logger.info("***** Running evaluation on split: %s %s *****", data_split, prefix)
        truth, predicted, guids, best_acc = [], [], [], []
        f = open(os.path.join(args.output_dir, "output_order.txt"), "w")
        multiref = False
        steps = 0
        model.eval()
        for batch in loader:
            tru = batch[3]
            if tru.ndim > 2:
                tru = tru[0].tolist()
                multiref = True
            else:
                tru = tru.view(-1).tolist()
            truth.append(tru)
            with torch.no_grad():
                inputs = {"input_ids": batch[0], "attention_mask": batch[1], "labels": batch[3]}
                if inputs["labels"].ndim > 2:
                    inputs["labels"] = inputs["labels"][:, 0, :]
                if getattr(args, "multimodal", False):
                    inputs["images"] = batch[-1]
                    if getattr(args, "include_num_img_regional_features", False):
                        inputs["img_regional_features"] = batch[-2]
                if len(tru) == 1 and not multiref:
                    pred = tru
                else:
                    pred = pointer_network(args, model, tokenizer, inputs)
            guids.append(str(batch[4][0]).split("###")[0])
            predicted.append(pred)
            print("{}|||{}".format(" ".join(map(str, pred)), " ".join(map(str, truth[-1]))),
                  file=f)
            steps += 1
            if getattr(args, "max_eval_steps", 0) > 0 and steps >= args.max_eval_steps:
                logger.info("Early stopping evaluation at step: %d", args.max_eval_steps)
                break
        accs, pmr, taus = cal_result(truth, predicted, best_acc, f, args=args)
        results["acc_dev"], results["pmr_dev"], results["taus_dev"] = accs, pmr, taus
        if getattr(args, "eval_save_all_results", False):
            with open(os.path.join(args.output_dir, "all_predictions.csv"), "w") as cf:
                w = csv.DictWriter(cf, fieldnames=["url"] + list(_CSV_METRICS))
                w.writeheader()
                for c in range(len(predicted)):
                    row = {k: compute_metrics(args, m, [predicted[c]], [truth[c]])
                           for k, m in _CSV_METRICS.items()}
                    row["url"] = guids[c]
                    w.writerow(row)
        out_file = os.path.join(out_dir, prefix, f"eval_results_split_{data_split}.txt")
        os.makedirs(os.path.dirname(out_file), exist_ok=True)
        with open(out_file, "w") as wr:
            for k in sorted(results):
                wr.write("%s = %s\n" % (k, str(results[k])))
        with open(os.path.join(args.output_dir, "all_eval_results.txt"), "a") as fh:
            fh.write(prefix)
            for k in sorted(results):
                fh.write("%s = %s\n" % (k, str(results[k])))
    return results
