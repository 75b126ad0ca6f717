"""md2hip -- MI355X-native hot path of the Monodepth2.jl training step.

Host-side mirror of the reference's Julia API (``Params``, ``TrainCache``, ``Model``,
``ResidualNetwork``, ``DepthDecoder``, ``PoseDecoder``, ``train_loss``, ``eval_disparity``,
``ADAM``) over the C-ABI of ``libmd2hip.so`` (include/md2.h).  There is no CPU fallback: every
op runs the HIP kernels and a missing library raises."""
from ._lib import MD2Error, lib  # noqa: F401
from .loss import Params, TrainCache, depth10k_intrinsics, loss_tail, pack_poses  # noqa: F401
from .model import (ADAM, DepthDecoder, Model, Pose, PoseDecoder, ResidualNetwork, ResNet,  # noqa: F401
                    disparity_bins, eval_disparity, flux_params, gradient, param_table, pullback, set_flux_params,
                    train_loss, train_step)
from .slow_depth import SlowDepth, adam_update, slow_depth  # noqa: F401
from .checkpoint import load_checkpoint, save_checkpoint  # noqa: F401
from .data import DataLoader, DChain, Depth10k, FlipX, KittyDataset, find_static  # noqa: F401
from .mpi import MPIDepthDecoder, mpi_forward  # noqa: F401

__all__ = ["Params", "TrainCache", "depth10k_intrinsics", "loss_tail", "pack_poses", "lib", "MD2Error",
           "ADAM", "DepthDecoder", "Model", "Pose", "PoseDecoder", "ResidualNetwork", "ResNet",
           "disparity_bins", "eval_disparity", "flux_params", "gradient", "param_table", "pullback", "set_flux_params", "train_loss",
           "train_step",
           "SlowDepth", "adam_update", "slow_depth", "load_checkpoint", "save_checkpoint",
           "DataLoader", "DChain", "Depth10k", "FlipX", "KittyDataset", "find_static",
           "MPIDepthDecoder", "mpi_forward"]
