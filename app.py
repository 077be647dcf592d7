"""Polyp segmentation inference app -- reference ``app.py:20-398`` (a Streamlit GUI).

Streamlit / plotly / OpenCV are not installable here, so the same application logic is exposed as
(1) a CLI (images, image folders, or frame folders / GIFs as "video") and (2) an HTTP service on
FastAPI + uvicorn (``python app.py --serve``; POST raw image bytes to ``/predict`` -> blended PNG, GET
``/metrics`` -> the PerformanceTracker table).  If streamlit IS importable, ``streamlit run app.py``
shows the same controls as the reference.

Behaviour kept from the reference: smp ``Unet`` + ``resnet50`` by default (``--model``/``--encoder``
override); ``num_class`` detected from the checkpoint head (``segmentation_head.0.weight`` or
``seg_head.weight``); non-strict load dropping unknown keys; Resize(320) + ImageNet Normalize;
sigmoid > 0.5 when ``num_class == 1`` else argmax; colour overlay blended 0.7/0.3; timing stats
(mean/min/max/std ms) for preprocessing, inference and visualisation.  Checkpoints are read with
``torch.load(weights_only=True)``.  On MI355X the native models run on the fused HIP executor.
"""

import argparse
import io
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image

from medical_segmentation_pytorch_amd.configs import MyConfig
from medical_segmentation_pytorch_amd.models import get_model
from medical_segmentation_pytorch_amd.utils.transforms import normalize_to_tensor, resize


class PerformanceTracker:
    def __init__(self):
        self.inference_times, self.preprocessing_times, self.visualization_times = [], [], []

    def add_inference_time(self, t):
        self.inference_times.append(t)

    def add_preprocessing_time(self, t):
        self.preprocessing_times.append(t)

    def add_visualization_time(self, t):
        self.visualization_times.append(t)

    @staticmethod
    def _stats(v):
        v = np.asarray(v if v else [0.0]) * 1000
        return [float(v.mean()), float(v.min()), float(v.max()), float(v.std())]

    def get_metrics_dataframe(self):
        data = {'Metric': ['Average', 'Minimum', 'Maximum', 'Standard Deviation'],
                'Inference Time (ms)': self._stats(self.inference_times),
                'Preprocessing Time (ms)': self._stats(self.preprocessing_times),
                'Visualization Time (ms)': self._stats(self.visualization_times)}
        try:
            import pandas as pd
            return pd.DataFrame(data)
        except Exception:   # pragma: no cover
            return data

    def plot_time_distribution(self, path=None):
        """Text box-plot summary (plotly is unavailable); returns the per-series quantiles."""
        out = {}
        for name, v in (('inference', self.inference_times), ('preprocessing', self.preprocessing_times),
                        ('visualization', self.visualization_times)):
            a = np.asarray(v if v else [0.0]) * 1000
            out[name] = {q: float(np.percentile(a, p)) for q, p in (('p5', 5), ('p25', 25), ('p50', 50),
                                                                     ('p75', 75), ('p95', 95))}
        if path:
            with open(path, 'w') as f:
                json.dump(out, f, indent=1)
        return out


class PolyPredictorApp:
    def __init__(self, model_path=None, model='smp', encoder='resnet50', decoder='unet', base_channel=None,
                 size=320, colormap_path=None, device=None):
        self.config = MyConfig()
        self.config.is_testing = True
        self.performance_tracker = PerformanceTracker()
        self.config.model, self.config.encoder, self.config.decoder = model, encoder, decoder
        self.config.encoder_weights = None
        if base_channel is not None:
            self.config.base_channel = base_channel
        model_path = model_path or self.config.model_path
        state_dict = None
        if model_path and os.path.isfile(model_path):
            ckpt = torch.load(model_path, map_location='cpu', weights_only=True)
            state_dict = ckpt['state_dict'] if isinstance(ckpt, dict) and 'state_dict' in ckpt else ckpt
            heads = [k for k in state_dict if 'segmentation_head.0.weight' in k or 'seg_head.weight' in k]
            self.config.num_class = state_dict[heads[0]].shape[0] if heads else 1
        else:
            print(f'[app] checkpoint {model_path!r} not found: random weights', file=sys.stderr)
        self.config.num_channel = 3
        self.device = device or torch.device('cuda' if torch.cuda.is_available() else 'cpu')
        self.model = get_model(self.config).to(self.device)
        if state_dict is not None:
            own = self.model.state_dict()
            state_dict = {k: v for k, v in state_dict.items() if k in own and own[k].shape == v.shape}
            self.model.load_state_dict(state_dict, strict=False)
        self.model.eval()
        self.forward = self.model
        if self.device.type == 'cuda':
            from medical_segmentation_pytorch_amd.utils.parallel import FusedModel, use_fused
            self.config.engine = 'auto'
            if use_fused(self.config, self.model, self.device):
                self.forward = FusedModel(self.model).eval()
        self.size = size
        self.colormap = None
        if colormap_path and os.path.exists(colormap_path):
            with open(colormap_path) as f:
                self.colormap = json.load(f)
        if self.colormap is None:
            self.colormap = self.generate_default_colormap()

    def generate_default_colormap(self):
        colors = [(255, 0, 0), (0, 255, 0), (0, 0, 255), (255, 255, 0), (255, 0, 255), (0, 255, 255)]
        return {str(i): list(c) for i, c in enumerate(colors[:max(self.config.num_class, 2)])}

    def preprocess_image(self, image):
        t0 = time.time()
        arr = np.array(image.convert('RGB'))
        arr = resize(arr, self.size, self.size, 'bilinear')
        x = normalize_to_tensor(arr).unsqueeze(0).to(self.device)
        self.performance_tracker.add_preprocessing_time(time.time() - t0)
        return x

    @torch.no_grad()
    def predict(self, input_tensor):
        t0 = time.time()
        pred = self.forward(input_tensor)
        if self.device.type == 'cuda':
            torch.cuda.synchronize()
        self.performance_tracker.add_inference_time(time.time() - t0)
        if self.config.num_class > 1:
            return torch.softmax(pred, 1).argmax(1).squeeze(0).cpu().numpy().astype(np.uint8)
        return (torch.sigmoid(pred).squeeze().cpu().numpy() > 0.5).astype(np.uint8)

    def visualize_prediction(self, original_image, mask):
        t0 = time.time()
        img = np.array(original_image.convert('RGB'))
        m = torch.from_numpy(mask)[None, None].float()
        m = F.interpolate(m, size=img.shape[:2], mode='nearest')[0, 0].numpy().astype(np.uint8)
        color = np.zeros_like(img)
        if self.config.num_class > 1:
            for c in np.unique(m):
                if c > 0:
                    color[m == c] = self.colormap.get(str(int(c)), [255, 0, 0])
        else:
            color[m == 1] = [255, 0, 0]
        blended = (img.astype(np.float32) * 0.7 + color.astype(np.float32) * 0.3).round().clip(0, 255).astype(np.uint8)
        self.performance_tracker.add_visualization_time(time.time() - t0)
        return blended

    def process_image(self, image):
        mask = self.predict(self.preprocess_image(image))
        return mask, self.visualize_prediction(image, mask)

    def process_video(self, frames, out_path=None, fps=10):
        """``frames``: a GIF path, a directory of frames, or an iterable of PIL images.  Writes an
        animated GIF (no video encoder is available) and returns the blended frames."""
        if isinstance(frames, str):
            if os.path.isdir(frames):
                frames = [Image.open(os.path.join(frames, f)) for f in sorted(os.listdir(frames))]
            else:
                gif = Image.open(frames)
                seq = []
                try:
                    while True:
                        seq.append(gif.copy().convert('RGB'))
                        gif.seek(gif.tell() + 1)
                except EOFError:
                    pass
                frames = seq
        out = [Image.fromarray(self.process_image(fr)[1]) for fr in frames]
        if out_path and out:
            out[0].save(out_path, save_all=True, append_images=out[1:], duration=int(1000 / fps), loop=0)
        return out

    def run(self, inputs, out_dir):
        os.makedirs(out_dir, exist_ok=True)
        for p in inputs:
            if os.path.isdir(p):
                self.run([os.path.join(p, f) for f in sorted(os.listdir(p))], out_dir)
                continue
            if p.lower().endswith('.gif'):
                self.process_video(p, os.path.join(out_dir, os.path.basename(p)))
                continue
            mask, blended = self.process_image(Image.open(p))
            stem = os.path.splitext(os.path.basename(p))[0]
            Image.fromarray(blended).save(os.path.join(out_dir, f'{stem}_blend.png'))
            Image.fromarray((mask * (255 if self.config.num_class == 1 else 1)).astype(np.uint8)).save(
                os.path.join(out_dir, f'{stem}_mask.png'))
        return self.performance_tracker.get_metrics_dataframe()


def make_server(app: PolyPredictorApp):
    from fastapi import FastAPI, Request
    from fastapi.responses import JSONResponse, Response
    api = FastAPI(title='MI355X polyp segmentation')

    @api.post('/predict')
    async def predict(request: Request):
        # raw image bytes in the body (multipart parsing needs python-multipart, not installed)
        image = Image.open(io.BytesIO(await request.body()))
        _, blended = app.process_image(image)
        buf = io.BytesIO()
        Image.fromarray(blended).save(buf, format='PNG')
        return Response(buf.getvalue(), media_type='image/png')

    @api.get('/metrics')
    def metrics():
        df = app.performance_tracker.get_metrics_dataframe()
        return JSONResponse(df.to_dict(orient='list') if hasattr(df, 'to_dict') else df)

    return api


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('inputs', nargs='*')
    ap.add_argument('--model-path', default=None)
    ap.add_argument('--model', default='smp')
    ap.add_argument('--encoder', default='resnet50')
    ap.add_argument('--decoder', default='unet')
    ap.add_argument('--base-channel', type=int, default=None)
    ap.add_argument('--out', default='app_out')
    ap.add_argument('--serve', action='store_true')
    ap.add_argument('--port', type=int, default=8000)
    a = ap.parse_args(argv)
    app = PolyPredictorApp(a.model_path, a.model, a.encoder, a.decoder, a.base_channel)
    if a.serve:
        import uvicorn
        uvicorn.run(make_server(app), host='127.0.0.1', port=a.port)
        return
    print(app.run(a.inputs, a.out))


if __name__ == '__main__':
    main()
