"""Figures of the solution and the trajectories (jaxsrc/utils/utils_plot.py, used by run_example.py:296-393).

Same figures as the reference (phi over (t, x) or x-y slices at a few times, each alp component, their sum,
trajectory plots), written as PNG files; TensorBoard image summaries are not supported.  Imported only when
--plot is given (needs matplotlib; the Agg backend, no display).
"""
import os

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402


def plot_solution_1d(phi, x_arr, t_arr, title=""):
    """utils_plot.py:11-41: phi [nt, nx] as a (t, x) colour map."""
    fig = plt.figure()
    x = np.asarray(x_arr).reshape(-1)
    t = np.asarray(t_arr).reshape(-1)
    plt.contourf(x, t, np.asarray(phi), 50)
    plt.colorbar()
    plt.xlabel("x")
    plt.ylabel("t")
    if title:
        plt.title(title)
    return fig


def plot_solution_2d(phi, x_arr, t_arr, T_divisor=4, title="", num_cols=2):
    """utils_plot.py:43-77: phi [nt, nx, ny] at T_divisor + 1 evenly spaced times."""
    phi = np.asarray(phi)
    nt = phi.shape[0]
    idx = sorted(set(int(round(k * (nt - 1) / T_divisor)) for k in range(T_divisor + 1)))
    rows = (len(idx) + num_cols - 1) // num_cols
    fig, axes = plt.subplots(rows, num_cols, figsize=(4 * num_cols, 3.5 * rows), squeeze=False)
    x = np.asarray(x_arr)[0, :, 0, 0]
    y = np.asarray(x_arr)[0, 0, :, 1]
    t = np.asarray(t_arr).reshape(-1)
    for k, ax in enumerate(axes.reshape(-1)):
        if k >= len(idx):
            ax.axis("off")
            continue
        c = ax.contourf(x, y, phi[idx[k]].T, 50)
        fig.colorbar(c, ax=ax)
        ax.set_title("t = {:.3f}".format(t[idx[k]]))
    if title:
        fig.suptitle(title)
    return fig


def plot_traj_1d(traj, t_arr, title=""):
    """utils_plot.py:79-89: traj [nt, n_samples] against t."""
    fig = plt.figure()
    plt.plot(np.asarray(t_arr).reshape(-1), np.asarray(traj))
    plt.xlabel("t")
    if title:
        plt.title(title)
    return fig


def plot_traj_2d(traj, title=""):
    """utils_plot.py:91-102: traj [nt, n_samples, 2] in the x-y plane."""
    traj = np.asarray(traj)
    fig = plt.figure()
    plt.plot(traj[:, :, 0], traj[:, :, 1])
    plt.xlabel("x")
    plt.ylabel("y")
    if title:
        plt.title(title)
    return fig


def save_fig(fig, filename, foldername=None):
    """utils_plot.py:104-112 without TensorBoard: <foldername>/<filename>.png."""
    path = os.path.join(foldername, filename) if foldername else filename
    fig.savefig(path + ".png")
    plt.close(fig)
    return path + ".png"


def plot_solution_figs(phi, alp, x_arr, t_arr, ndim, egno, n_ctrl, folder):
    """run_example.py:296-334: phi, every alp component and their sum."""
    num_cols = 1 if egno == 3 else 2
    t = np.asarray(t_arr)
    plot = plot_solution_1d if ndim == 1 else (lambda f, x, tt: plot_solution_2d(f, x, tt, num_cols=num_cols))
    save_fig(plot(phi, x_arr, t), "phi", folder)
    names = ["alp_1", "alp_2"] if ndim == 1 else ["alp_11", "alp_12", "alp_21", "alp_22"]
    for i in range(2 ** ndim):
        save_fig(plot(alp[i, ..., 0], x_arr, t[:-1]), names[i] + "_x", folder)
        if n_ctrl == 2:
            save_fig(plot(alp[i, ..., 1], x_arr, t[:-1]), names[i] + "_y", folder)
    alp_sum = np.sum(alp, axis=0)
    save_fig(plot(alp_sum[..., 0], x_arr, t[:-1]), "alp_sum_x", folder)
    if n_ctrl == 2:
        save_fig(plot(alp_sum[..., 1], x_arr, t[:-1]), "alp_sum_y", folder)


def plot_traj_figs(traj_x, traj_alp, t, ndim, egno, n_ctrl, folder):
    """run_example.py:360-393: trajectory figures."""
    if egno == 3:
        save_fig(plot_traj_1d(traj_x[..., 0], t), "traj_vel", folder)
        save_fig(plot_traj_1d(traj_x[..., 1], t), "traj_pos", folder)
        save_fig(plot_traj_1d(traj_alp[..., 0], t[:-1]), "traj_acc", folder)
        return
    save_fig(plot_traj_1d(traj_x, t) if ndim == 1 else plot_traj_2d(traj_x), "traj_x", folder)
    if n_ctrl == 1:
        save_fig(plot_traj_1d(traj_alp[..., 0], t[:-1]), "traj_alp", folder)
    else:
        save_fig(plot_traj_2d(traj_alp), "traj_alp", folder)
