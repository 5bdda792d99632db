"""Host-side evaluation with the semantics of the reference's EvaluationFuncs.py.

These run on the probabilities the engine returns (B, 2, Ncr) against the one-hot
labels (B, 2, Ncr), exactly as model_2.train/test call them, quirks included
(SURVEY Appendix B.9):
  * top_ACC        EvaluationFuncs.py:27-37   argmax agreement over all relations
                   (np.argmax: ties pick class 0)
  * prec/recall/f1 EvaluationFuncs.py:79-106  np.ceil of labels AND probabilities,
                   then sklearn on channel 0 (so every prediction is 1)
  * AUC            EvaluationFuncs.py:108-153 resets auc inside the graph loop and
                   returns the LAST graph's AUC over the number of scored graphs
  * process_edge   EvaluationFuncs.py:11-16   identity
The correct-count of top_ACC is also exposed (top_acc_count) so data-parallel ranks
can all-reduce it instead of gathering probabilities.
"""
import numpy as np


def process_edge(Ra):
    return Ra


def top_acc_count(label, probs):
    """Number of relations whose argmax class agrees (numpy argmax tie rule)."""
    label = np.asarray(label)
    probs = np.asarray(probs)
    return int((np.argmax(probs, axis=1) == np.argmax(label, axis=1)).sum())


def top_ACC(label, probs):
    label = np.asarray(label)
    return float(top_acc_count(label, probs) / (label.shape[0] * label.shape[2]))


def _per_graph(score_fn, label, real):
    labelz = np.ceil(np.asarray(label))
    realz = np.ceil(np.asarray(real))
    acc = 0.0
    for i in range(labelz.shape[0]):
        acc += score_fn(labelz[i, 0, :], realz[i, 0, :])
    return acc / labelz.shape[0]


def prec(label, real):
    from sklearn.metrics import precision_score
    return _per_graph(precision_score, label, real)


def recall(label, real):
    from sklearn.metrics import recall_score
    return _per_graph(recall_score, label, real)


def f1(label, real):
    from sklearn.metrics import f1_score
    return _per_graph(f1_score, label, real)


def AUC(label, real):
    from sklearn.metrics import roc_auc_score
    label = np.asarray(label)
    real = np.asarray(real)
    auc, count = 0.0, 0
    for i in range(label.shape[0]):
        auc, count = 0.0, 0                      # reset per graph (reference behaviour)
        lab_idx = np.argmax(label[i], axis=0)    # class index of each relation
        pos = np.argmin(label[i], axis=0)        # channel whose score is used
        score = np.where(pos == 0, real[i, 0], real[i, 1])
        try:
            s = roc_auc_score(lab_idx, score)
        except ValueError:
            print("ValueError: Only one class present in y_true. ROC AUC score is not "
                  "defined in that case.")
        else:
            auc += s
            count += 1
    return auc / count
