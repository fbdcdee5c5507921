"""ola_log_tiled_kernel (csrc/fdlp_misc.hip) takes the output row of element q of a tile as
(int)((q + 0.5f) * (1.0f / B)) instead of q / B.  The float quotient must equal the integer one for every
q < kOlaRows * B the kernel sees; float32 arithmetic here rounds like the kernel's v_add/v_mul_f32."""
import numpy as np

K_OLA_ROWS = 32


def test_float_reciprocal_row_index_is_exact():
    for B in range(1, 1025):
        q = np.arange(K_OLA_ROWS * B, dtype=np.int64)
        inv_b = np.float32(1.0) / np.float32(B)
        t = ((q.astype(np.float32) + np.float32(0.5)) * inv_b).astype(np.int64)
        assert np.array_equal(t, q // B), B
