"""ToyDiskDataset (dataset.py of the reference): loads `<name>*_{train,val,test}.npz` files
holding {train,val,test}_data -> dict(start_image, start_state, image, state, q, visible).

The reference stores states as float64 (create_dataset.py:131); they are cast to float32
here (the particle path computes in fp32).  The npz holds a pickled dict,
so it is read with allow_pickle=True: only load files your own generator wrote.
"""
import os

import numpy as np
import torch
from torch.utils.data import Dataset


class ToyDiskDataset(Dataset):
    KEYS = ("start_image", "start_state", "image", "state", "q", "visible")

    def __init__(self, data_path, filename, datatype="train_data"):
        self.data_path, self.filename = data_path, filename
        files = sorted(os.listdir(data_path))
        tag = {"train_data": "train", "val_data": "val"}.get(datatype, "test")
        chosen = [os.path.join(data_path, f) for f in files if f.startswith(filename) and tag in f]
        self.train_data = [os.path.join(data_path, f) for f in files if f.startswith(filename) and "train" in f]
        self.val_data = [os.path.join(data_path, f) for f in files if f.startswith(filename) and "val" in f]
        self.test_data = [os.path.join(data_path, f) for f in files if f.startswith(filename) and "test" in f]
        data = dict(np.load(chosen[0], allow_pickle=True))[datatype].item()  # first file only (:38-39)
        for k in self.KEYS:
            v = np.asarray(data[k])
            if v.dtype == np.float64:
                v = v.astype(np.float32)
            setattr(self, k, v)
        self.data_size = len(self.start_image)
        print(self.data_size)

    def __len__(self):
        return self.data_size

    def __getitem__(self, idx):
        if torch.is_tensor(idx):
            idx = idx.tolist()
        return tuple(getattr(self, k)[idx] for k in self.KEYS)
