"""MI355X-native CWT episode engine (drop-in for the episodic forward / inner-adapt path of
TeamOfProfGuo/Few_Shot_Seg_CWT).  See DESIGN.md.

Reference-shaped entry points:
  get_model(args).extract_features(x)             src/model/pspnet.py:15,172
  MultiHeadAttentionOne(n_head, 512, 512, 512)    src/model/transformer.py:33
  intersectionAndUnionGPU / batch_...             src/util.py:237,280
  validate_transformer / do_epoch                 src/test.py:103, src/train.py:166
  get_train_loader / get_val_loader, EpisodicData src/dataset/dataset.py:17-117,180-327
  checkpoint.load_backbone / *_transformer_checkpoint   src/train.py:57-75,147-163; src/test.py:61-89
  CosCls / get_classifier / get_corr              src/model/pspnet.py:290-334, model_util.py:101-109
"""
from .pspnet import PSPNet, get_model  # noqa: F401
from .transformer import MultiHeadAttentionOne  # noqa: F401
from .util import AverageMeter, batch_intersectionAndUnionGPU, intersectionAndUnionGPU  # noqa: F401
from .optimizer import HipSGD, get_optimizer  # noqa: F401
from .episode import (EpisodeEngine, SyntheticEpisodes, do_epoch, inner_adapt,  # noqa: F401
                      validate_transformer)
from .dataset import EpisodicData, get_train_loader, get_val_loader  # noqa: F401
from . import checkpoint  # noqa: F401
from .heads import CosCls, get_classifier, get_corr, parse_param_coscls  # noqa: F401

__version__ = "0.1.0"
