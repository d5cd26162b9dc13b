"""The product's host entropy tables (dcvc_amd/entropy.py) equal the
reference's own tables (golden fixtures built by the reference's
GaussianEncoder/BitEstimator.update + ops.cpp)."""
import numpy as np

from dcvc_amd.entropy import ScaleTable, FactorizedTable


def _eq(ours, ref):
    c, l, o = ref
    np.testing.assert_array_equal(ours.cdf, c)
    np.testing.assert_array_equal(ours.sizes.reshape(-1), l.reshape(-1))
    np.testing.assert_array_equal(ours.offsets.reshape(-1), o.reshape(-1))


def test_scale_tables(dc_golden):
    _eq(ScaleTable("gaussian"), dc_golden.table("i_y"))
    _eq(ScaleTable("laplace"), dc_golden.table("p_y"))


def test_factorized_tables(dc_golden):
    isd, psd = dc_golden.i_state_dict(), dc_golden.p_state_dict()
    _eq(FactorizedTable(isd, "bit_estimator_z", 256), dc_golden.table("i_z"))
    _eq(FactorizedTable(psd, "bit_estimator_z", 128), dc_golden.table("p_z"))
    _eq(FactorizedTable(psd, "bit_estimator_z_mv", 64), dc_golden.table("p_mvz"))
