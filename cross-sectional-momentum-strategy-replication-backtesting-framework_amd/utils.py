"""Host-side performance summary, identical to the reference's src/utils.py:5-21."""
from __future__ import annotations

import os

import numpy as np


def ensure_dir(path):
    """src/utils.py:5-6."""
    os.makedirs(path, exist_ok=True)


def sharpe(returns, freq_per_year=252):
    """Annualised Sharpe ratio, src/utils.py:8-16 (NumPy on the host: a handful of values)."""
    rs = np.array(returns)
    if len(rs) == 0:
        return float("nan")
    mean = rs.mean() * freq_per_year
    sd = rs.std(ddof=1) * (freq_per_year ** 0.5)
    if sd == 0:
        return float("nan")
    return mean / sd


def save_plot(fig, path):
    """src/utils.py:18-21."""
    import matplotlib.pyplot as plt

    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)
