"""Native Criteo preprocessor vs the line-by-line Python definition."""
import numpy as np
import pytest

from cloudtik_amd.data.criteo import (dense_transform, parse_criteo, parse_criteo_reference,
                                      write_synthetic_criteo)


@pytest.mark.parametrize("max_ind_range", [-1, 1000])
def test_native_parser_matches_reference(tmp_path, max_ind_range):
    p = tmp_path / "day.tsv"
    write_synthetic_criteo(str(p), 3000, seed=1)
    got = parse_criteo(str(p), max_ind_range, threads=7)
    ref = parse_criteo_reference(str(p), max_ind_range)
    for k in ("y", "X_int", "X_cat", "counts"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    assert (got["counts"] <= (1000 if max_ind_range > 0 else 3000)).all()


def test_parser_handles_no_trailing_newline_and_empty(tmp_path):
    p = tmp_path / "x.tsv"
    p.write_text("1\t" + "\t".join(["5"] * 13) + "\t" + "\t".join(["a"] * 26))
    d = parse_criteo(str(p))
    assert d["y"].tolist() == [1] and d["X_int"][0].tolist() == [5] * 13 and d["counts"].tolist() == [1] * 26
    e = tmp_path / "empty.tsv"
    e.write_text("")
    assert parse_criteo(str(e))["y"].shape == (0,)


def test_dense_transform():
    np.testing.assert_allclose(dense_transform(np.array([[-3, 0, 1, 9]], np.int32)),
                               np.log1p(np.array([[0, 0, 1, 9]], np.float32)))


def test_cli(tmp_path):
    from cloudtik_amd.data.criteo import main
    p = tmp_path / "day.tsv"
    write_synthetic_criteo(str(p), 200)
    main(["--raw-data-file", str(p), "--processed-data-file", str(tmp_path / "out.npz")])
    d = np.load(tmp_path / "out.npz")
    assert d["X_cat"].shape == (200, 26) and d["counts"].shape == (26,)
