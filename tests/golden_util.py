"""Helpers to read the committed reference fixtures (tests/golden/*.npz).

The fixtures were produced by tools/gen_golden.py from the real reference
compiled in place (oracle/_ref/libsblas_ref.so); they hold only data.
"""
from __future__ import annotations

import glob
import os
from dataclasses import dataclass, field

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@dataclass
class Run:
    m: int
    lda: int
    ldc: int
    alpha: float
    beta: float
    a: np.ndarray
    c: np.ndarray
    out: np.ndarray


@dataclass
class Case:
    name: str
    rows: int
    cols: int
    stride: int
    trans: bool
    table_size: int
    dm: np.ndarray
    table: np.ndarray
    s_rows: int
    s_cols: int
    pos: np.ndarray
    val: np.ndarray
    panel_row_off: np.ndarray
    panel_col_off: np.ndarray
    panel_begin: np.ndarray
    panel_end: np.ndarray
    copyto: dict = field(default_factory=dict)     # trans -> (stride, array)
    runs: list = field(default_factory=list)

    def dense_b(self) -> np.ndarray:
        """B = S^T as a dense (s_cols x s_rows) float matrix, from the index rule."""
        T = self.table_size
        dm = self.dm.reshape(self.rows, self.stride)[:, : self.cols]
        tab = np.zeros(256, np.float32)
        tab[:T] = self.table[:T]
        live = dm < T
        d = np.where(live, tab[dm], np.float32(0)).astype(np.float32)
        # NoTrans: S = dm (rows x cols) so B = dm^T; Trans: S = dm^T so B = dm
        return d if self.trans else np.ascontiguousarray(d.T)

    def live_mask_b(self) -> np.ndarray:
        dm = self.dm.reshape(self.rows, self.stride)[:, : self.cols]
        live = dm < self.table_size
        return live if self.trans else np.ascontiguousarray(live.T)


def _load(path: str) -> Case:
    z = np.load(path, allow_pickle=False)
    c = Case(
        name=os.path.basename(path)[:-4], rows=int(z["rows"]), cols=int(z["cols"]),
        stride=int(z["stride"]), trans=bool(int(z["trans"])), table_size=int(z["table_size"]),
        dm=z["dm"], table=z["table"], s_rows=int(z["s_rows"]), s_cols=int(z["s_cols"]),
        pos=z["pos"], val=z["val"], panel_row_off=z["panel_row_off"],
        panel_col_off=z["panel_col_off"], panel_begin=z["panel_begin"],
        panel_end=z["panel_end"])
    if "copyto_notrans" in z.files:
        c.copyto[False] = (int(z["copyto_notrans_stride"]), z["copyto_notrans"])
        c.copyto[True] = (int(z["copyto_trans_stride"]), z["copyto_trans"])
    for i in range(int(z["n_runs"])):
        c.runs.append(Run(int(z[f"r{i}_m"]), int(z[f"r{i}_lda"]), int(z[f"r{i}_ldc"]),
                          float(z[f"r{i}_alpha"]), float(z[f"r{i}_beta"]), z[f"r{i}_a"],
                          z[f"r{i}_c"], z[f"r{i}_out"]))
    return c


def case_paths() -> list[str]:
    return sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(p).startswith("kernels"))


def case_names() -> list[str]:
    return [os.path.basename(p)[:-4] for p in case_paths()]


def load_case(name: str) -> Case:
    return _load(os.path.join(GOLDEN, name + ".npz"))


def load_kernels() -> dict:
    z = np.load(os.path.join(GOLDEN, "kernels.npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def bits_equal(x: np.ndarray, y: np.ndarray) -> bool:
    """Bit-exact fp32 equality (NaN payloads included)."""
    x = np.ascontiguousarray(x, np.float32).reshape(-1)
    y = np.ascontiguousarray(y, np.float32).reshape(-1)
    return x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))
