"""eval.py result formats (pertrenderer_amd.results): the writers produce
the file names and json.dump text of experiments/eval.py:566-573 / :644-661, the np.save
curves and image grid of :394-405 / :787-821; the reader and run comparison round-trip."""
import json

import numpy as np
import pytest

from pertrenderer_amd import results as R

TABLES = dict(
    mean_errors={"gaussian": [12.5, 3.25], "softras": [20.0, 8.5]},
    final_errors={"gaussian": [[1.0, 2.0], [3.0, 4.0]], "softras": [[5.0], [6.0]]},
    init_errors={"gaussian": [[90.0, 80.0]], "softras": [[90.0]]},
    var_errors={"gaussian": [1.5, 0.5], "softras": [2.0, 1.0]},
    mean_solved={"gaussian": {"5": [0.5, 0.75], "10": [0.75, 1.0]}, "softras": {"5": [0.25, 0.5], "10": [0.5, 0.5]}},
    params={"lr-smoothing-MC": [[0.05, 1e-3, 1e-2, 8]], "lr": [0.05], "sigma": [1e-3], "gamma": [1e-2], "MC": [8],
            "adapt_params": [[1.0, 1.0]]},
    exp_setup={"nb_iter": 200, "image_size": 256},
)


def test_pose_tables_match_eval_py_files(tmp_path):
    R.write_pose_results(tmp_path, **TABLES)
    for key, name in R.POSE_FILES.items():
        # eval.py:648-661: open(path_res / name, 'w'); json.dump(table, file)
        assert (tmp_path / name).read_text() == json.dumps(TABLES[key])
    assert R.read_results(tmp_path) == TABLES


def test_runtime_tables_and_numpy_scalars(tmp_path):
    rt = {"gaussian": [np.float32(0.5), np.float64(0.25)], "softras": [0.125]}
    mem = {"gaussian": [np.int64(1024)], "softras": [2048]}
    R.write_runtime_results(tmp_path, rt, mem)
    assert (tmp_path / "runtimes.txt").read_text() == json.dumps({"gaussian": [0.5, 0.25], "softras": [0.125]})
    assert json.loads((tmp_path / "memory.txt").read_text()) == {"gaussian": [1024], "softras": [2048]}


def test_results_dir_follows_eval_py(tmp_path):
    assert R.results_dir(7, cwd=tmp_path / "experiments") == tmp_path / "experiments/results/7"


def test_optimization_details_and_grid(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    imgs = np.random.default_rng(0).uniform(-0.5, 1.5, (6, 8, 8, 4)).astype(np.float32)
    d = R.write_optimization_details(tmp_path / "res", [3.0, 2.0, 1.0], [0.5, 0.25, 0.125], imgs,
                                     datenow="2026-01-01-00:00:00")
    got = R.read_optimization_details(d)
    np.testing.assert_array_equal(got["loss_values"], [3.0, 2.0, 1.0])
    np.testing.assert_array_equal(got["gradient_values"], [0.5, 0.25, 0.125])
    png = d / "grid_cube.png"
    assert png.read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"
    assert imgs.min() < 0  # the caller's images are not clipped in place by the grid


def test_image_grid_requires_rows_and_cols_together(tmp_path):
    with pytest.raises(ValueError):
        R.image_grid(np.zeros((2, 4, 4, 4)), tmp_path, rows=2)


def test_compare_pose_results():
    b = json.loads(json.dumps(TABLES))
    b["mean_errors"]["gaussian"][1] += 0.5
    b["mean_solved"]["softras"]["10"][0] -= 0.25
    rep = R.compare_pose_results(TABLES, b)
    assert rep["gaussian"]["max_abs_mean_error_diff"] == pytest.approx(0.5)
    assert rep["gaussian"]["max_abs_solved_diff"] == 0.0
    assert rep["softras"]["solved_diff"]["10"] == pytest.approx([-0.25, 0.0])
    assert R.compare_pose_results(TABLES, TABLES)["softras"]["max_abs_mean_error_diff"] == 0.0
