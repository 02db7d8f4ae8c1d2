"""Dataset peek (reference path load_data.py:1-16): shape, head and class counts, read through
the native CSV reader."""
import os

import numpy as np

from fraud_detection_amd.data.io import read_table

if __name__ == "__main__":
    X, y, names = read_table(os.getenv("DATA_CSV", "data/creditcard.csv"))
    print("shape:", (X.shape[0], X.shape[1] + 1))
    print("columns:", names + ["Class"])
    print("head:\n", np.round(X[:5], 4))
    if y is not None:
        print("class counts:", dict(zip(*np.unique(y, return_counts=True))))
