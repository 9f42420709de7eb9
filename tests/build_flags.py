"""Which build of libgeneralsparse the tests run against.  The experiments build
(make -C generalsparse_amd/csrc exp, loaded with GS_LIBRARY=.../libgeneralsparse_exp.so)
adds the kernels measured slower and kept opt-in; their tests skip in the default build."""
import pytest

import generalsparse_amd as gsa

EXPERIMENTS = gsa.get_config("GS_EXPERIMENTS") == 1
experiments = pytest.mark.skipif(not EXPERIMENTS, reason="experiments-build kernel (GS_LIBRARY=libgeneralsparse_exp.so)")


def need_experiments(flag=True):
    if flag and not EXPERIMENTS:
        pytest.skip("experiments-build kernel (GS_LIBRARY=libgeneralsparse_exp.so)")
