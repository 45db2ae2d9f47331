"""Generate tests/golden/prf.json: sklearn.metrics.precision_recall_fscore_support(
average="binary", zero_division=1) on key / sustain activation vectors, the call the
reference's MidiEvaluationWrapper makes once per step (robopianist/wrappers/evaluation.py:
135-140, 162-164).

scikit-learn is the reference's own dependency (setup.py pins 1.4.2; this image has 1.7.2:
both compute P = tp/(tp+fp), R = tp/(tp+fn) and, since 1.3, F = 2tp/(|true| + |pred|), with
zero_division replacing 0/0). Runs anywhere sklearn is importable; the fixture is committed.

Usage: python tests/golden/make_eval_golden.py
"""
import json
import warnings
from pathlib import Path

import numpy as np
import sklearn
from sklearn.metrics import precision_recall_fscore_support

OUT = Path(__file__).resolve().parent / "prf.json"


def main():
    warnings.simplefilter("ignore")
    rng = np.random.RandomState(2024)
    cases = []
    edge = [(np.zeros(88), np.zeros(88)), (np.eye(88)[3], np.zeros(88)), (np.zeros(88), np.eye(88)[5]),
            (np.ones(88), np.ones(88)), (np.ones(88), np.zeros(88)), (np.zeros(88), np.ones(88))]
    for n in (1, 1, 1, 1):
        edge.append((rng.randint(0, 2, n).astype(float), rng.randint(0, 2, n).astype(float)))
    edge += [(np.array([a], float), np.array([b], float)) for a in (0, 1) for b in (0, 1)]
    for p_true, p_pred in ((0.05, 0.05), (0.1, 0.3), (0.02, 0.0), (0.0, 0.02), (0.5, 0.5)):
        for _ in range(8):
            edge.append(((rng.rand(88) < p_true).astype(float), (rng.rand(88) < p_pred).astype(float)))
    for yt, yp in edge:
        p, r, f, _ = precision_recall_fscore_support(y_true=yt, y_pred=yp, average="binary", zero_division=1)
        cases.append({"y_true": yt.astype(int).tolist(), "y_pred": yp.astype(int).tolist(),
                      "prf": [float(p), float(r), float(f)]})
    OUT.write_text(json.dumps({"sklearn": sklearn.__version__, "cases": cases}))
    print(f"wrote {OUT}: {len(cases)} cases")


if __name__ == "__main__":
    main()
