"""Every example notebook in notebooks/ runs top to bottom (the reference ships one notebook per
algorithm). CPU path here; the ``gpu`` variant runs the same cells on the HIP kernels."""
import glob
import json
import os

import pytest

NB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "notebooks")
NOTEBOOKS = sorted(glob.glob(os.path.join(NB_DIR, "*.ipynb")))


def _run(path):
    nb = json.load(open(path))
    ns = {"__name__": "__notebook__"}
    for cell in nb["cells"]:
        if cell["cell_type"] == "code":
            exec(compile("".join(cell["source"]), path, "exec"), ns)  # noqa: S102 - our own notebooks


@pytest.mark.parametrize("path", NOTEBOOKS, ids=[os.path.basename(p) for p in NOTEBOOKS])
def test_notebook_runs_cpu(path, monkeypatch):
    monkeypatch.setenv("SRML_FORCE_CPU", "1")
    _run(path)


@pytest.mark.gpu
@pytest.mark.parametrize("path", NOTEBOOKS, ids=[os.path.basename(p) for p in NOTEBOOKS])
def test_notebook_runs_gpu(path, monkeypatch):
    monkeypatch.delenv("SRML_FORCE_CPU", raising=False)
    _run(path)
