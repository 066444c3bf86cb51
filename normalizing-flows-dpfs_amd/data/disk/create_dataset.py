"""Synthetic disk-tracking dataset (data/disk/create_dataset.py of the reference): a red disc
of radius 7 on a 128 x 128 frame with coloured distractor discs, all moving under a spring /
drag process model with Gaussian position noise.  Same ToyExample class, methods, process
model, numpy-RNG draw order, 80/10/10 split and npz layout
(`<name><index>_{train,val,test}.npz` holding {train,val,test}_data -> dict(start_image,
start_state, image, state, q, visible)), so dataset.ToyDiskDataset reads either.

    python create_dataset.py --out-dir ./data/disk --num-examples 1000 --sequence-length 50

The reference rasterises the discs with OpenCV (cv2.circle, filled), which is not part of this
build: ``fill_circle`` fills the pixels whose centres lie within the radius (a disc of radius
7 covers 149 pixels, as cv2's does).  Images are therefore not pinned to the reference's
pixel for pixel; the trajectories (states, q) are -- the RNG draws are identical
(tests/test_dataset.py against the reference's own process model).
"""
import argparse
import logging
import os
import sys

import numpy as np


def fill_circle(im, center, radius, color):
    """Filled disc: every pixel (x, y) with (x - cx)^2 + (y - cy)^2 <= r^2 (integer centre as
    cv2's, x = column, y = row); clipped to the frame."""
    cx, cy = int(center[0]), int(center[1])
    h, w = im.shape[:2]
    y0, y1 = max(cy - radius, 0), min(cy + radius + 1, h)
    x0, x1 = max(cx - radius, 0), min(cx + radius + 1, w)
    if y0 >= y1 or x0 >= x1:
        return im
    yy, xx = np.mgrid[y0:y1, x0:x1]
    m = (xx - cx) ** 2 + (yy - cy) ** 2 <= radius * radius
    im[y0:y1, x0:x1][m] = color
    return im


class ToyExample():
    def __init__(self, param):
        self.im_size = param.width
        self.out_dir = param.out_dir
        self.name = param.name
        self.num_examples = param.num_examples
        self.sequence_length = param.sequence_length
        self.file_size = min(self.num_examples, param.file_size)
        self.spring_force = 0.1
        self.drag_force = 0.0075
        self.cols = [(0, 255, 0), (0, 0, 255), (0, 255, 255), (255, 0, 255), (255, 255, 0), (255, 255, 255)]
        os.makedirs(self.out_dir, exist_ok=True)
        self.log = logging.getLogger(param.name)
        self.log.setLevel(logging.DEBUG)
        if not self.log.handlers:
            ch = logging.StreamHandler(sys.stdout)
            ch.setLevel(logging.DEBUG)
            ch.setFormatter(logging.Formatter('%(asctime)s: [%(name)s] [%(levelname)s] %(message)s'))
            self.log.addHandler(ch)

    def create_dataset(self, num_distractors, pos_noise):
        self.keys = ['start_image', 'start_state', 'image', 'state', 'q', 'visible']
        data = {key: [] for key in self.keys}
        self.log.info('Starting to generate dataset ' + self.name)
        counts = np.zeros(3, dtype=np.int64)
        ct, index = 0, 0
        while counts[0] < self.num_examples:
            values = self._get_data(num_distractors, pos_noise)
            ct += 1
            for key in self.keys:
                data[key] += [values[key]]
            if len(data['image']) >= self.file_size:
                counts += self._save(data, index)
                index += 1
                data = {key: [] for key in self.keys}
            if ct % 250 == 0:
                self.log.info('Done ' + str(ct) + ' of ' + str(int(self.num_examples / 0.8)))
        if len(data['image']) > 0:
            counts += self._save(data, index)
        with open(os.path.join(self.out_dir, 'info_' + self.name + '.txt'), 'w') as fi:
            fi.write('Num data points: ' + str(int(counts.sum())) + '\n')
            fi.write('Num train: ' + str(int(counts[0])) + '\n')
            fi.write('Num val: ' + str(int(counts[1])) + '\n')
            fi.write('Num test: ' + str(int(counts[2])) + '\n')
        self.log.info('Done')

    def _get_data(self, num_distractors, pos_noise):
        """One sequence: initial disc and distractor draws, then per step the process model
        for the disc and each distractor (create_dataset.py:120-171, same draw order)."""
        half = self.im_size // 2
        pos = np.random.uniform(-half, half, size=(2))
        vel = np.random.normal(loc=0, scale=1, size=(2)) * 3
        initial_state = np.array([pos[0], pos[1], vel[0], vel[1]])
        distractors = []
        for _ in range(num_distractors):
            pos = np.random.uniform(-half, half, size=(2))
            vel = np.random.normal(loc=0, scale=1, size=(2)) * 3
            rad = np.random.choice(np.arange(3, 10))
            col = np.random.choice(len(self.cols))
            distractors += [(rad, np.array([pos[0], pos[1], vel[0], vel[1]]), col)]
        initial_im, _ = self._observation_model(initial_state, distractors)
        states, images, qs, rs = [], [], [], []
        last_state = initial_state
        for _ in range(self.sequence_length):
            state, q = self._process_model(last_state, pos_noise)
            distractors = [(d[0], self._process_model(d[1], pos_noise)[0], d[2]) for d in distractors]
            im, vis = self._observation_model(state, distractors)
            states += [state]
            images += [im]
            qs += [q]
            rs += [vis]
            last_state = state
        return {'start_image': initial_im, 'start_state': initial_state, 'image': np.array(images),
                'state': np.array(states), 'q': np.array(qs), 'visible': np.array(rs)}

    def _observation_model(self, state, distractors):
        im = np.zeros((self.im_size, self.im_size, 3))
        half = self.im_size // 2
        fill_circle(im, (state[0] + half, state[1] + half), 7, (255, 0, 0))
        for d in distractors:
            fill_circle(im, (d[1][0] + half, d[1][1] + half), d[0], self.cols[d[2]])
        # visible pixels of the red disc (it may be covered by distractors or leave the frame)
        mask = (im[:, :, 0] == 255) & (im[:, :, 1] == 0) & (im[:, :, 2] == 0)
        return im.astype(np.float32) / 255., np.sum(mask)

    def _process_model(self, state, pos_noise):
        """Spring pull to the centre, quadratic drag, N(0, pos_noise^2) position noise
        (create_dataset.py:197-216); q = the noise scales [pos, pos, 2, 2]."""
        new_state = np.copy(state)
        pull_force = - self.spring_force * state[:2]
        drag_force = - self.drag_force * state[2:] ** 2 * np.sign(state[2:])
        new_state[0] += state[2]
        new_state[1] += state[3]
        new_state[2] += pull_force[0] + drag_force[0]
        new_state[3] += pull_force[1] + drag_force[1]
        new_state[:2] += np.random.normal(loc=0, scale=pos_noise, size=(2))
        new_state[2:] += 0.0
        return new_state, np.array([pos_noise, pos_noise, 2., 2.])

    def _save(self, data, index=0):
        """Shuffle, split 80/10/10 and write <name><index>_{train,val,test}.npz."""
        length = len(data['image'])
        permutation = np.random.permutation(length)
        data = {key: np.copy(np.asarray(data[key]))[permutation] for key in self.keys}
        train_size = int(np.floor(length * 8. / 10.))
        val_size = int(np.floor(length * 1. / 10.))
        test_size = length - train_size - val_size
        bounds = {'train': (0, train_size), 'val': (train_size, train_size + val_size),
                  'test': (train_size + val_size, length)}
        for split, (a, b) in bounds.items():
            if b > a:
                part = {key: np.copy(data[key][a:b]) for key in self.keys}
                np.savez(os.path.join(self.out_dir, self.name + str(index) + f"_{split}.npz"), **{split + "_data": part})
        return np.array([train_size, val_size, test_size])


def main(argv=None):
    parser = argparse.ArgumentParser('toy datset')
    parser.add_argument('--name', dest='name', type=str, default='toy')
    parser.add_argument('--out-dir', dest='out_dir', type=str, default='./TwentyfiveDistractors')
    parser.add_argument('--sequence-length', dest='sequence_length', type=int, default=50)
    parser.add_argument('--width', dest='width', type=int, default=128)
    parser.add_argument('--num-examples', dest='num_examples', type=int, default=1000)
    parser.add_argument('--file-size', dest='file_size', type=int, default=500)
    parser.add_argument('--pos-noise', dest='pos_noise', type=float, default=2.0)
    parser.add_argument('--num-distractors', dest='num_distractors', type=int, default=25)
    args = parser.parse_args(argv)
    args.name = args.name + '_pn=' + str(args.pos_noise) + '_d=' + str(args.num_distractors) + '_const'
    if not os.path.exists(os.path.join(args.out_dir, 'info_' + args.name + '.txt')):
        ToyExample(args).create_dataset(args.num_distractors, args.pos_noise)
    else:
        print('name already exists')


if __name__ == "__main__":
    main()
