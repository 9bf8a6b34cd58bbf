"""Learner registry — the reference's eight learners (PipelineMap.scala:68) + extension.

Reference factory: MLNodeGenerator maps a request to (worker, PS) nodes carrying an
mlAPI learner (omldm/utils/generators/MLNodeGenerator.scala:20-76); here a request's
``learner.name`` selects one of these classes.
"""
from omldm_amd.models.base import Learner, RoundContext
from omldm_amd.models.dense import HT, NN, ORR, KMeans, MultiClassPA
from omldm_amd.models.linear import PA, SVM, LogisticRegression, RegressorPA
from omldm_amd.models.preprocess import (PREPROCESSORS, MinMaxScaler, PolynomialFeatures,
                                         Preprocessor, StandardScaler, make_preprocessor)

LEARNERS = {
    "PA": PA,
    "RegressorPA": RegressorPA,
    "ORR": ORR,
    "SVM": SVM,
    "MultiClassPA": MultiClassPA,
    "K-means": KMeans,
    "NN": NN,
    "HT": HT,
    "LogisticRegression": LogisticRegression,
}


def make_learner(name: str, hyper: dict | None, space, device) -> Learner:
    if name not in LEARNERS:
        raise KeyError(f"unknown learner {name!r}")
    return LEARNERS[name](hyper, space, device)


__all__ = ["LEARNERS", "make_learner", "Learner", "RoundContext", "PREPROCESSORS",
           "make_preprocessor", "Preprocessor", "StandardScaler", "MinMaxScaler",
           "PolynomialFeatures"]
