#!/usr/bin/env python3
"""Disease prediction application: vision + NLP ensemble (reference
applications/ai/disease_prediction: ``train.py`` runs DLSA (a BERT classifier over the
radiology report), a vision classifier over the contrast-enhanced mammogram and a
"consult" step that combines both models' class probabilities).

Pipeline on the MI355X modeling library:
  1. prepare   -- patient table (report text + image + label), stratified train/test split
  2. dlsa      -- BERT text classifier fine-tuned on the reports   (modeling.transfer_learning)
  3. vision    -- ResNet image classifier fine-tuned on the images (modeling.transfer_learning)
  4. consult   -- learns the per-class ensemble weight w_c on held-out VALIDATION predictions
                  (p = w_c * p_text + (1 - w_c) * p_vision, grid search maximising macro F1;
                  the reference fits on training outputs, which fine-tuned models overfit),
                  then predicts the test split; writes model (weights) + predictions + metrics.

Without ``--data`` it synthesises patients: each class has a characteristic vocabulary in
the report and a characteristic texture/colour in the image, with label noise chosen so
that neither modality alone is perfect.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

CLASSES = ["Normal", "Benign", "Malignant"]
WORDS = {
    "Normal": "no suspicious enhancement symmetric tissue unremarkable stable".split(),
    "Benign": "circumscribed oval mass fibroadenoma cyst smooth margins".split(),
    "Malignant": "spiculated irregular mass heterogeneous enhancement architectural distortion".split(),
}
FILLER = "the patient study images breast left right views were obtained and compared with prior".split()


def synthetic_patients(n: int, image_size: int = 64, seed: int = 0):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 3, n)
    # each modality sees a corrupted label for a different 25% of the patients
    y_text = np.where(rng.random(n) < 0.25, rng.integers(0, 3, n), y)
    y_img = np.where(rng.random(n) < 0.25, rng.integers(0, 3, n), y)
    texts = []
    for c in y_text:
        words = list(rng.choice(FILLER, 12)) + list(rng.choice(WORDS[CLASSES[c]], 4))
        rng.shuffle(words)
        texts.append(" ".join(words))
    centers = np.array([[0.8, -0.4, 0.0], [-0.5, 0.7, -0.2], [0.0, -0.3, 0.9]], np.float32)[:, :, None, None]
    imgs = centers[y_img] + 0.9 * rng.normal(size=(n, 3, image_size, image_size)).astype(np.float32)
    return texts, imgs, y


def split(n, test_fraction, seed):
    idx = np.random.default_rng(seed).permutation(n)
    k = int(n * (1 - test_fraction))
    return idx[:k], idx[k:]


def macro_f1(y, pred, k=3):
    f1s = []
    for c in range(k):
        tp = np.sum((pred == c) & (y == c))
        fp = np.sum((pred == c) & (y != c))
        fn = np.sum((pred != c) & (y == c))
        f1s.append(0.0 if tp == 0 else 2 * tp / (2 * tp + fp + fn))
    return float(np.mean(f1s))


def run_dlsa(texts, y, tr, te, args, device):
    from cloudtik_amd.modeling.transfer_learning.datasets import HashTokenizer, TextClassificationDataset
    from cloudtik_amd.modeling.transfer_learning.text_classification import TextClassificationModel
    tok = HashTokenizer(vocab_size=args.vocab, max_length=32)
    m = TextClassificationModel(args.text_model, num_classes=3, device=device, classes=CLASSES,
                                vocab_size=args.vocab)
    ds = TextClassificationDataset([texts[i] for i in tr], y[tr].tolist(), tok)
    m.train(ds, epochs=args.epochs, batch_size=32, lr=args.text_lr, log_every=0)

    def probs(idx):
        ids, mask = tok([texts[i] for i in idx])
        with torch.no_grad():
            return m.predict(ids, mask).cpu().numpy()
    return probs(tr), probs(te)


def run_vision(imgs, y, tr, te, args, device):
    from cloudtik_amd.modeling.transfer_learning.datasets import ArrayImageDataset
    from cloudtik_amd.modeling.transfer_learning.image_classification import ImageClassificationModel
    m = ImageClassificationModel(args.image_model, num_classes=3, freeze_backbone=False, device=device,
                                 classes=CLASSES)
    m.train(ArrayImageDataset(imgs[tr], y[tr]), epochs=args.epochs, batch_size=32, lr=args.image_lr)

    def probs(idx):
        out = []
        for s in range(0, len(idx), 128):
            x = torch.from_numpy(imgs[idx[s:s + 128]])
            with torch.no_grad():
                out.append(torch.softmax(m.predict(x).float(), -1).cpu().numpy())
        return np.concatenate(out)
    return probs(tr), probs(te)


class Consult:
    """Per-class convex combination of the two models' probabilities."""

    def __init__(self, grid=np.linspace(0.0, 1.0, 21)):
        self.grid = grid
        self.w = np.full(3, 0.5)

    def combine(self, pt, pv):
        return self.w * pt + (1 - self.w) * pv

    def fit(self, pt, pv, y):
        for _ in range(2):                         # coordinate ascent over the classes
            for c in range(3):
                best, best_w = -1.0, self.w[c]
                for w in self.grid:
                    self.w[c] = w
                    f = macro_f1(y, self.combine(pt, pv).argmax(1))
                    if f > best + 1e-12:
                        best, best_w = f, w
                self.w[c] = best_w
        return self

    def save(self, path):
        with open(path, "w") as f:
            f.write("class,text_weight\n" + "".join(f"{c},{w:.4f}\n" for c, w in zip(CLASSES, self.w)))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--patients", type=int, default=1200)
    ap.add_argument("--test-fraction", type=float, default=0.25)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--text-model", default="bert-tiny")
    ap.add_argument("--image-model", default="resnet_tiny")
    ap.add_argument("--vocab", type=int, default=4096)
    ap.add_argument("--text-lr", type=float, default=2e-3)
    ap.add_argument("--image-lr", type=float, default=1e-3)
    ap.add_argument("--output-dir", default="")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    torch.manual_seed(args.seed)
    device = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    texts, imgs, y = synthetic_patients(args.patients, seed=args.seed)
    tr, te = split(len(y), args.test_fraction, args.seed)
    nv = max(1, len(tr) // 5)
    va, tr = tr[:nv], tr[nv:]                      # validation split for the consult step
    ev = np.concatenate([va, te])
    pt_tr, pt_ev = run_dlsa(texts, y, tr, ev, args, device)
    pv_tr, pv_ev = run_vision(imgs, y, tr, ev, args, device)
    pt_va, pt_te, pv_va, pv_te = pt_ev[:nv], pt_ev[nv:], pv_ev[:nv], pv_ev[nv:]
    consult = Consult().fit(pt_va, pv_va, y[va])
    pred = consult.combine(pt_te, pv_te).argmax(1)
    res = {"dlsa_f1": macro_f1(y[te], pt_te.argmax(1)), "vision_f1": macro_f1(y[te], pv_te.argmax(1)),
           "ensemble_f1": macro_f1(y[te], pred), "text_weights": consult.w.round(3).tolist(),
           "test_patients": int(len(te)), "device": str(device)}
    if args.output_dir:
        os.makedirs(args.output_dir, exist_ok=True)
        consult.save(os.path.join(args.output_dir, "consult-model.csv"))
        with open(os.path.join(args.output_dir, "predictions.json"), "w") as f:
            json.dump({"patients": te.tolist(), "predicted": [CLASSES[i] for i in pred],
                       "label": [CLASSES[i] for i in y[te]]}, f)
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
