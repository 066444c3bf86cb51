"""Command-line flags: the reference's arguments.py surface (arguments.py:5-103), unchanged,
plus build-only flags for the MI355X path:

  --rng-mode {device,host}   device: Philox on the GPU (default); host: the reference's
                             CPU-generator draws uploaded each step (parity mode)
  --force-resample           resample every step (the ESS gate is then bypassed)
  --NF-dyn-flow {RealNVP,MAF} dynamic flow family (MAF is BASELINE config 4; not wired
                             in the reference)
"""
import argparse


def build_parser():
    p = argparse.ArgumentParser()
    a = p.add_argument
    a("--gpu", action="store_false", help="whether to use GPU")
    a("--gpu-index", type=int, default=0, help="index num of GPU to use")
    a("--trainType", dest="trainType", type=str, default="DPF", choices=["DPF", "SDPF", "UDPF"],
      help="train type: supervised, semi, unsupervised learning")
    a("--pretrain_ae", action="store_true", help="pretrain of autoencoder model")
    a("--pretrain-NFcond", action="store_true", help="pretrain of conditional normalising flow model")
    a("--e2e-train", action="store_false", help="End to end training")
    a("--load-pretrainModel", action="store_true", help="Load pretrain model")
    a("--NF-dyn", action="store_true", help="train using normalising flow")
    a("--NF-cond", action="store_true", help="train using conditional normalising flow")
    a("--measurement", type=str, default="cos", help="|CRNVP|cos|NN|CGLOW|gaussian|")
    a("--NF-lr", type=float, default=2.5, help="NF learning rate")
    a("--epsilon", type=float, default=0.1, help="epsilon in OT resampling")
    a("--scaling", type=float, default=0.75, help="scaling in OT resampling")
    a("--alpha", type=float, default=0.5, help="hyperparameter for soft resampling")
    a("--threshold", type=float, default=1e-3, help="threshold in OT resampling")
    a("--max_iter", type=int, default=100, help="max iterarion in OT resampling")
    a("--resampler_type", type=str, default="ot", help="|ot|soft|")
    a("--resume", action="store_true", help="resume training from checkpoint")
    a("--Dyn_nn", action="store_true", help="learned dynamic model using neural network")
    a("--Obs_feature", action="store_false", help="Compute likelihood using feature similarity")
    a("--batchsize", type=int, default=32, help="batch size")
    a("--hiddensize", type=int, default=32, help="hidden size")
    a("--lr", type=float, default=1e-4, help="learning rate")
    a("--optim", type=str, default="Adam", help="type of optim")
    a("--num-epochs", type=int, default=500, help="num epochs")
    a("--num-particles", type=int, default=100, help="num of particles")
    a("--split-ratio", type=float, default=0.9, help="split training data")
    a("--labeledRatio", type=float, default=1.0, help="labeled training data")
    a("--init-with-true-state", action="store_true",
      help="init_with_true_state, default: false, uniform initialisation")
    a("--dropout-keep-ratio", type=float, default=0.3, help="1-dropout_ratio")
    a("--particle_std", type=float, default=0.2, help="particle std")
    a("--seed", type=int, default=2, help="random seed")
    a("--sequence-length", dest="sequence_length", type=int, default=50, help="length of the generated sequences")
    a("--width", dest="width", type=int, default=128, help="width (= height) of the generated observations")
    a("--pos-noise", dest="pos_noise", type=float, default=20.0, help="sigma for the positional process noise")
    a("--vel-noise", dest="vel_noise", type=float, default=20.0, help="sigma for the velocity noise")
    a("--true-pos-noise", dest="true_pos_noise", type=float, default=2.0,
      help="sigma for the positional process noise when generating datasets")
    a("--true-vel-noise", dest="true_vel_noise", type=float, default=2.0,
      help="sigma for the velocity noise when generating datasets")
    a("--block-length", dest="block_length", type=int, default=10, help="block length for pseudo-likelihood")
    a("--testing", action="store_true", help="Check testing performance")
    a("--model-path", type=str, default="./model/e2e_model_bestval_e2e.pth", help="path of saved model")
    a("--x_size", type=tuple, default=(3, 8, 8))
    a("--y_size", type=tuple, default=(3, 8, 8))
    a("--x_hidden_channels", type=int, default=8)
    a("--x_hidden_size", type=int, default=16)
    a("--y_hidden_channels", type=int, default=8)
    a("-K", "--flow_depth", type=int, default=1)
    a("-L", "--num_levels", type=int, default=1)
    a("--learn_top", type=bool, default=False)
    a("--x_bins", type=float, default=256.0)
    a("--y_bins", type=float, default=256.0)
    a("--individual", action="store_true", help="set individual opimizers for different units")
    # build-only (MI355X path)
    a("--rng-mode", dest="rng_mode", choices=["device", "host"], default="device",
      help="device: Philox on the GPU; host: the reference CPU-generator draws (parity mode)")
    a("--force-resample", dest="force_resample", action="store_true", help="resample at every step")
    a("--NF-dyn-flow", dest="NF_dyn_flow", choices=["RealNVP", "MAF"], default="RealNVP",
      help="dynamic flow family")
    return p


def parse_args(args=None):
    return build_parser().parse_args(args)
