"""mini_gym_learn/utils (rsl_rl's trajectory helpers; the recurrent-policy path the reference never takes)."""
import torch


def split_and_pad_trajectories(tensor, dones):
    """[T, N, ...] -> trajectories split at the dones, zero-padded to the longest, [L, n_traj, ...], and the mask of
    their valid steps [L, n_traj]."""
    dones = dones.clone()
    dones[-1] = 1
    flat_dones = dones.transpose(1, 0).reshape(-1, 1)
    ends = torch.cat((flat_dones.new_tensor([-1], dtype=torch.int64), flat_dones.nonzero()[:, 0]))
    lengths = ends[1:] - ends[:-1]
    trajs = torch.split(tensor.transpose(1, 0).flatten(0, 1), lengths.tolist())
    padded = torch.nn.utils.rnn.pad_sequence(trajs)
    masks = lengths > torch.arange(0, tensor.shape[0], device=tensor.device).unsqueeze(1)
    return padded, masks


def unpad_trajectories(trajectories, masks):
    """Inverse of split_and_pad_trajectories."""
    return trajectories.transpose(1, 0)[masks.transpose(1, 0)].view(
        -1, trajectories.shape[0], trajectories.shape[-1]).transpose(1, 0)
