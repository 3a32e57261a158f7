"""Result persistence and plots (src/utils/visualization.py:14-112).

save_results writes the same JSON the reference writes.  Plotting is outside the
hot path; the two plot helpers draw with matplotlib when it is importable and
otherwise only report that no figure was made."""
from __future__ import annotations

import json
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np


def _plain(obj):
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    if isinstance(obj, dict):
        return {k: _plain(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_plain(v) for v in obj]
    if isinstance(obj, np.integer):
        return int(obj)
    if isinstance(obj, np.floating):
        return float(obj)
    return obj


def save_results(results: Dict, filepath: str):
    """JSON dump with NumPy values converted, parent directories created."""
    path = Path(filepath)
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w") as f:
        json.dump(_plain(results), f, indent=2)


def _pyplot():
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        return plt
    except Exception:  # noqa: BLE001 - plotting is optional
        return None


def plot_ber_curves(snr_db: np.ndarray, ber_data: Dict[str, List[float]], title: str = "BER vs SNR",
                    save_path: Optional[str] = None, show_plot: bool = True):
    plt = _pyplot()
    if plt is None:
        print("matplotlib not available: no figure for %s" % title)
        return
    plt.figure(figsize=(10, 6))
    for label, ber in ber_data.items():
        plt.semilogy(snr_db, ber, marker="o", label=label, linewidth=2, markersize=6)
    plt.xlabel("SNR (dB)")
    plt.ylabel("Bit Error Rate (BER)")
    plt.title(title)
    plt.grid(True, which="both", alpha=0.3)
    plt.legend()
    plt.tight_layout()
    if save_path:
        plt.savefig(save_path, dpi=150, bbox_inches="tight")
    plt.close()


def plot_comparison(data: Dict[str, float], ylabel: str = "Value", title: str = "Performance Comparison",
                    save_path: Optional[str] = None, show_plot: bool = True):
    plt = _pyplot()
    if plt is None:
        print("matplotlib not available: no figure for %s" % title)
        return
    plt.figure(figsize=(8, 6))
    plt.bar(list(data.keys()), list(data.values()), alpha=0.7)
    plt.ylabel(ylabel)
    plt.title(title)
    plt.grid(True, axis="y", alpha=0.3)
    plt.tight_layout()
    if save_path:
        plt.savefig(save_path, dpi=150, bbox_inches="tight")
    plt.close()
