"""CPU restatement of ``metrics.calculate_mAP`` (metrics.py:8-145) — TEST INFRASTRUCTURE ONLY.

VOC 11-point mAP, restated in numpy/torch-CPU with the reference's arithmetic:
  * per class c (1..C-1), detections of class c sorted by score, descending (:74).  The
    reference's ``torch.sort`` is not stable; this restatement breaks ties by input order
    (stable), which is what the HIP path does — fixtures use tie-free scores;
  * each detection, in that order, takes the max IoU (``find_jaccard_overlap``: +1e-5
    denominator and the zero-size masks, :99) over the class-c objects of its image, first
    index on ties (:100); no object in the image -> false positive (:92-94);
  * ``max_overlap.item() > threshold`` compares the float32 IoU as a Python float (:108);
    a difficult matched object yields neither TP nor FP (:110), an undetected easy one a TP
    (marked detected, :112-114), an already detected one an FP (:116-117), no match an FP;
  * cumulative TP/FP in float32, precision = tp / (tp + fp + 1e-10), recall = tp / n_easy
    (:121-125); for t in float32 arange(0, 1.1, 0.1): max precision where recall >= t, else 0
    (:128-134); AP = mean of the 11 (float32); classes without detections keep AP 0 (:71-72);
  * mAP = mean of the C-1 APs (float32, :139).
"""
import numpy as np
import torch

from .match_ref import find_jaccard_overlap


def recall_thresholds():
    """torch.arange(0, 1.1, 0.1) exactly as the reference builds it (float32 values)."""
    return torch.arange(start=0, end=1.1, step=.1).numpy().astype(np.float32)


def calculate_map(det_boxes, det_labels, det_scores, true_boxes, true_labels, true_difficulties,
                  threshold, n_classes):
    """Lists of per-image numpy arrays -> (ap [C-1] float32, mAP float)."""
    B = len(det_boxes)
    t_img = np.concatenate([np.full(len(l), i, np.int64) for i, l in enumerate(true_labels)]) \
        if B else np.zeros(0, np.int64)
    t_box = np.concatenate([np.asarray(b, np.float32).reshape(-1, 4) for b in true_boxes])
    t_lab = np.concatenate([np.asarray(l, np.int64).reshape(-1) for l in true_labels])
    t_dif = np.concatenate([np.asarray(d, np.int64).reshape(-1) for d in true_difficulties])
    d_img = np.concatenate([np.full(len(l), i, np.int64) for i, l in enumerate(det_labels)])
    d_box = np.concatenate([np.asarray(b, np.float32).reshape(-1, 4) for b in det_boxes])
    d_lab = np.concatenate([np.asarray(l, np.int64).reshape(-1) for l in det_labels])
    d_sc = np.concatenate([np.asarray(s, np.float32).reshape(-1) for s in det_scores])
    thr_t = recall_thresholds()
    ap = np.zeros(n_classes - 1, np.float32)
    for c in range(1, n_classes):
        tm = t_lab == c
        tc_img, tc_box, tc_dif = t_img[tm], t_box[tm], t_dif[tm]
        n_easy = int((1 - tc_dif).sum())
        detected = np.zeros(len(tc_dif), np.uint8)
        dm = d_lab == c
        dc_img, dc_box, dc_sc = d_img[dm], d_box[dm], d_sc[dm]
        nd = len(dc_sc)
        if nd == 0:
            continue
        order = np.argsort(-dc_sc, kind='stable')
        dc_img, dc_box = dc_img[order], dc_box[order]
        tp = np.zeros(nd, np.float32)
        fp = np.zeros(nd, np.float32)
        for d in range(nd):
            sel = np.nonzero(tc_img == dc_img[d])[0]
            if len(sel) == 0:
                fp[d] = 1
                continue
            ov = find_jaccard_overlap(dc_box[d:d + 1], tc_box[sel])[0]
            ind = int(np.argmax(ov))
            if float(ov[ind]) > threshold:
                if tc_dif[sel[ind]] == 0:
                    if detected[sel[ind]] == 0:
                        tp[d] = 1
                        detected[sel[ind]] = 1
                    else:
                        fp[d] = 1
            else:
                fp[d] = 1
        ctp = np.cumsum(tp, dtype=np.float32)
        cfp = np.cumsum(fp, dtype=np.float32)
        with np.errstate(divide='ignore', invalid='ignore'):
            prec = ctp / (ctp + cfp + np.float32(1e-10))
            rec = ctp / np.float32(n_easy)
        pr = np.zeros(11, np.float32)
        for i, t in enumerate(thr_t):
            above = rec >= t
            pr[i] = prec[above].max() if above.any() else np.float32(0)
        ap[c - 1] = torch.from_numpy(pr).mean().item()
    return ap, float(torch.from_numpy(ap).mean().item())
