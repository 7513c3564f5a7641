"""CPU tests of the ml-side glue (sketchml_amd/gradient.py): toAuto's Java-int nnz rule
(DenseDoubleGradient.scala:92-95)."""
import pytest

from sketchml_amd.gradient import auto_dense


@pytest.mark.parametrize("nnz,dim,dense", [
    (67, 100, True),                                 # 100*2/3 = 66: 67 > 66 -> dense
    (66, 100, False),
    (0, 0, False),
    (1, 2, False),                                   # 2*2/3 = 1
    (2, 2, True),
    (700_000_000, 1_073_741_823, False),             # largest dim without wrap: limit 715,827,882
    (715_827_883, 1_073_741_823, True),
    (5, 1_073_741_824, True),                        # dim*2 wraps to -2^31: limit -715,827,882
])
def test_auto_dense_java_int(nnz, dim, dense):
    assert auto_dense(nnz, dim) is dense
