"""Model constants of the fingerprint QAP matcher.

Values follow the reference's module constants (``src/model/ngm.py:34-55``) and the
AFA-U encoder hyper-parameters (``src/model/afau.py:26-35``).
"""
import math

FEATURE_CHANNEL_NODE = 256          # ngm.py:34
FEATURE_CHANNEL_EDGE = 512          # ngm.py:35
NODE_FEATURE_DIM = 768              # ngm.py:36
GLOBAL_FEATURE_DIM = 512            # ngm.py:37
GLOBAL_STATE_DIM = 1024             # ngm.py:38

SK_TAU = 0.01                       # ngm.py:45
SK_EMB = 1                          # ngm.py:46
GNN_FEAT = (16, 16, 16)             # ngm.py:47
GNN_LAYER = 3                       # ngm.py:48
UNIV_SIZE = 600                     # ngm.py:52
SK_ITER_NUM = 10                    # ngm.py:53
SK_EPSILON = 1e-10                  # ngm.py:54
K_FACTOR = 50.0                     # ngm.py:55
GNN_SK_ITER = 20                    # PYGNNLayer default sk_iter (gnn.py:173/182)

SPLINE_KERNEL = 5                   # spline_conv.py:17  (kernel_size=5, dim=2, degree 1 open)
SPLINE_CELLS = SPLINE_KERNEL * SPLINE_KERNEL
RESCALE = (320.0, 240.0)            # Net.rescale, ngm.py:160 (feature_align's ori_size)
PSEUDO_RESCALE = 320.0              # gmdataset.py:36,171 (max(RESCALE))

AFAU_EMB = 600                      # afau.py:27
AFAU_EMB_PAD = 640                  # bf16 operand copies of 600-wide rows, K padded to a multiple of 64
AFAU_HEADS = 16                     # afau.py:28
AFAU_QKV = 16                       # afau.py:29
AFAU_FF = 256                       # afau.py:30
AFAU_MS_HIDDEN = 16                 # afau.py:31
AFAU_MS_INIT = 10.0                 # afau.py:32-33
AFAU_SQRT_QKV = math.sqrt(16)       # afau.py:34
REG_HIDDEN = 8                      # ngm.py:180-190

CLS_CHANNELS = (16, 32)             # ngm.py:85
BN_EPS = 1e-5
IN_EPS = 1e-5
