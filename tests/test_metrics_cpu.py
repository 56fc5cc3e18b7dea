"""Device-confusion metrics reproduce sklearn's macro scores (trainer.py:387-443)."""
import numpy as np
import pytest
from sklearn import metrics as skm

from vgan.metrics import scores


@pytest.mark.parametrize("seed", range(12))
def test_scores_match_sklearn(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 400))
    k_true = int(rng.integers(1, 8))
    y = rng.integers(0, k_true, n)
    p = np.where(rng.random(n) < 0.6, y, rng.integers(0, 7, n))
    conf = np.zeros((7, 7), dtype=np.int64)
    np.add.at(conf, (y, p), 1)
    f1, prec, rec, acc = scores(conf)
    kw = dict(average="macro", zero_division=0)
    assert f1 == pytest.approx(skm.f1_score(y, p, **kw), abs=1e-12)
    assert prec == pytest.approx(skm.precision_score(y, p, **kw), abs=1e-12)
    assert rec == pytest.approx(skm.recall_score(y, p, **kw), abs=1e-12)
    assert acc == pytest.approx(skm.accuracy_score(y, p), abs=1e-12)
