"""Tanner-graph / syndrome helpers with the reference's API (src/ldpc/utils.py:11-89)."""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def create_tanner_graph(H: np.ndarray) -> Tuple[List[List[int]], List[List[int]]]:
    """(var_neighbors, check_neighbors), ascending indices (utils.py:11-34)."""
    Hb = np.asarray(H) == 1
    checks = [list(np.nonzero(row)[0].astype(int)) for row in Hb]
    vars_ = [list(np.nonzero(col)[0].astype(int)) for col in Hb.T]
    return vars_, checks


def calculate_syndrome(H: np.ndarray, received: np.ndarray) -> np.ndarray:
    return (np.asarray(H) @ np.asarray(received)) % 2


def check_syndrome(H: np.ndarray, codeword: np.ndarray) -> bool:
    return bool(np.all(calculate_syndrome(H, codeword) == 0))


def count_errors(original: np.ndarray, decoded: np.ndarray) -> int:
    return int(np.sum(np.asarray(original) != np.asarray(decoded)))


hamming_distance = count_errors
