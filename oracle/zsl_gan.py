"""zsl_gan.py -- TEST INFRASTRUCTURE ONLY: oracle for the zero-shot GAN training step.

Only ``tests/`` import this module, as the checker. A torch restatement (float64 by
default, autograd for the gradients) of

* spectral normalisation (``module/spectral_norm.py:39-89``): in training mode one power
  iteration updates u, v in place under no_grad, then sigma = u . (W v) with u, v constants;
* the generator MLP of ``UnifiedModel.generate`` (``module/model.py:679-686``) and
  ``LayerNormalization`` (``module/submodule.py:58-77``);
* the ``Discriminator`` (``module/zsl_module.py:112-138``), ``calc_gradient_penalty``
  (``module/utils.py:692-707``) and one Discriminator step and one Generator step of
  ``ZSLmodule.train`` (``zsl_module.py:417-600``) with Adam (betas (0.5, 0.9)).

Parity status: unpinned by reference fixtures (none exist; running the reference's Python is
denied in this pipeline). Written from the reference's source text.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def sn_weight(w, u, v, train, eps=1e-12):
    """spectral_norm.compute_weight: returns (W / sigma, u, v) (u, v updated copies)."""
    if train:
        with torch.no_grad():
            v = F.normalize(torch.mv(w.t(), u), dim=0, eps=eps)
            u = F.normalize(torch.mv(w, v), dim=0, eps=eps)
    sigma = torch.dot(u, torch.mv(w, v))
    return w / sigma, u, v


def layer_norm_ref(z, a, b, eps=1e-3):
    if z.size(1) == 1:
        return z
    mu = z.mean(-1, keepdim=True)
    sd = z.std(-1, keepdim=True)
    return (z - mu) / (sd + eps) * a + b


def generator(noise, cls, layers, ln_a, ln_b, train):
    """layers: [(W_orig, b, u, v)] x 3 -> (out, [(u, v) after])."""
    x = torch.cat([noise, cls], 1)
    uv = []
    for (w, b, u, v) in layers:
        wn, u2, v2 = sn_weight(w, u, v, train)
        uv.append((u2, v2))
        x = F.linear(x, wn, b)
    return layer_norm_ref(x, ln_a, ln_b), uv


def discriminator(x, centroids, p, train):
    """Discriminator.forward (zsl_module.py:124-138); p: dict of fc_middle/fc_TF weight_orig,
    bias, u, v and layer_norm a_2, b_2. Returns (middle, logit, class_scores, new uv).
    fc_middle is CALLED twice per forward (:127 on the sample, :130 on the centroids), so in
    training mode its power iteration runs twice and the two calls use different sigmas."""
    wm, um, vm = sn_weight(p["fc_middle.weight_orig"], p["fc_middle.weight_u"], p["fc_middle.weight_v"], train)
    ln = lambda z: layer_norm_ref(z, p["layer_norm.a_2"], p["layer_norm.b_2"])
    mid = ln(F.leaky_relu(F.linear(x, wm, p["fc_middle.bias"])))
    wm2, um, vm = sn_weight(p["fc_middle.weight_orig"], um, vm, train)
    cen = ln(F.leaky_relu(F.linear(centroids, wm2, p["fc_middle.bias"])))
    wt, ut, vt = sn_weight(p["fc_TF.weight_orig"], p["fc_TF.weight_u"], p["fc_TF.weight_v"], train)
    logit = F.linear(mid, wt, p["fc_TF.bias"])
    return mid, logit, mid @ cen.t(), {"fc_middle": (um, vm), "fc_TF": (ut, vt)}


class GANRef:
    """Float64 restatement of one D step and one G step of ZSLmodule.train (zsl_module.py:
    419-600) with explicit tensors. D: dict name -> leaf tensor (weight_orig, bias, a_2, b_2) /
    buffer (weight_u, weight_v); G: (layers [(W, b, u, v)] x 3, ln_a, ln_b)."""

    def __init__(self, D, G, centroids, margin=5.0, gan_batch_rela=2, lr_D=1e-4, lr_G=1e-4, gp_lambda=10.0):
        self.D, self.G, self.centroids = D, G, centroids
        self.margin, self.gan_batch_rela, self.gp_lambda = margin, gan_batch_rela, gp_lambda
        self.d_params = [v for k, v in D.items() if not (k.endswith("weight_u") or k.endswith("weight_v"))]
        layers, a, b = G
        self.g_params = [t for (w, bb, _, _) in layers for t in (w, bb)] + [a, b]
        self.opt_D = torch.optim.Adam(self.d_params, lr=lr_D, betas=(0.5, 0.9))
        self.opt_G = torch.optim.Adam(self.g_params, lr=lr_G, betas=(0.5, 0.9))

    def _disc(self, x, train):
        mid, logit, cls, uv = discriminator(x, self.centroids, self.D, train)
        if train:
            for name, (u, v) in uv.items():
                self.D[name + ".weight_u"], self.D[name + ".weight_v"] = u, v
        return mid, logit, cls

    def _gen(self, cls_rows, noise, train):
        layers, a, b = self.G
        out, uv = generator(noise, cls_rows, layers, a, b, train)
        if train:
            self.G = ([(w, bb, u, v) for (w, bb, _, _), (u, v) in zip(layers, uv)], a, b)
        return out

    def d_step(self, cls_rows, real, neg, labels, noise, alpha):
        with torch.no_grad():
            fake = self._gen(cls_rows, noise, False)
        pick = lambda c: c[torch.arange(len(labels)), labels]
        _, real_dec, real_cls = self._disc(real, True)
        _, fake_dec, fake_cls = self._disc(fake, True)
        _, _, neg_cls = self._disc(neg, True)
        loss_real, loss_fake = -torch.mean(real_dec), torch.mean(fake_dec)
        loss_rela = F.relu(self.margin - (pick(real_cls) - pick(neg_cls))).mean()
        loss_fake_cls = F.relu(self.margin - (pick(fake_cls) - pick(neg_cls))).mean()
        inter = (alpha * real + (1 - alpha) * fake).requires_grad_(True)
        _, disc, _ = self._disc(inter, True)
        grads = torch.autograd.grad(disc, inter, torch.ones_like(disc), create_graph=True, retain_graph=True)[0]
        gp = ((grads.norm(2, dim=1) - 1) ** 2).mean() * self.gp_lambda
        loss = loss_real + 0.5 * loss_rela + loss_fake + gp + 0.5 * loss_fake_cls
        self.opt_D.zero_grad()
        loss.backward()
        grads = [p.grad.detach().clone() for p in self.d_params]
        self.opt_D.step()
        return torch.stack([loss, loss_real, loss_rela, loss_fake, loss_fake_cls]).detach(), grads

    def g_step(self, cls_rows, real, neg, labels, noise):
        pick = lambda c: c[torch.arange(len(labels)), labels]
        sample = self._gen(cls_rows, noise, True)
        _, dec, cls = self._disc(sample, False)
        _, _, real_cls = self._disc(real, False)
        _, _, neg_cls = self._disc(neg, False)
        loss_fake = -torch.mean(dec)
        loss_cls = F.relu(self.margin - (pick(cls) - pick(neg_cls))).mean()
        loss_real_cls = F.relu(self.margin - (pick(real_cls) - pick(neg_cls))).mean()
        vp = torch.zeros((), dtype=sample.dtype)
        for i in range(self.centroids.shape[0]):
            idx = (labels == i).nonzero().flatten()
            if len(idx):
                vp = vp + (sample[idx].mean(0) - self.centroids[i]).pow(2).sum().sqrt()
        vp = vp * (1.0 / self.gan_batch_rela)
        loss = loss_fake + loss_cls + 3.0 * vp
        self.opt_G.zero_grad()
        for p in self.d_params:
            p.grad = None
        loss.backward()
        grads = [p.grad.detach().clone() for p in self.g_params]
        self.opt_G.step()
        return torch.stack([loss, loss_fake, loss_cls, loss_real_cls, vp]).detach(), grads
