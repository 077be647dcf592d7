import os
import subprocess
import sys

import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_model_infos():
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'get_model_infos.py'), '--model', 'ducknet',
                          '--base_channel', '17'], capture_output=True, text=True, timeout=300, cwd='/tmp')
    assert '40.10M' in out.stdout and '93.22 GFLOP' in out.stdout


def test_app_cli_and_server(tmp_path):
    sys.path.insert(0, ROOT)
    from app import PolyPredictorApp, make_server
    from medical_segmentation_pytorch_amd.models import DuckNet
    m = DuckNet(1, 3, 4)
    torch.save({'state_dict': m.state_dict()}, tmp_path / 'ck.pth')
    app = PolyPredictorApp(str(tmp_path / 'ck.pth'), model='ducknet', base_channel=4, size=64,
                           device=torch.device('cpu'))
    assert app.config.num_class == 1                 # detected from seg_head.weight
    img = Image.fromarray((np.random.rand(50, 70, 3) * 255).astype(np.uint8))
    img.save(tmp_path / 'a.jpg')
    frames = [img, img]
    frames[0].save(tmp_path / 'v.gif', save_all=True, append_images=frames[1:])
    df = app.run([str(tmp_path / 'a.jpg'), str(tmp_path / 'v.gif')], str(tmp_path / 'out'))
    assert os.path.isfile(tmp_path / 'out' / 'a_blend.png') and os.path.isfile(tmp_path / 'out' / 'v.gif')
    assert len(app.performance_tracker.inference_times) >= 2
    from fastapi.testclient import TestClient
    client = TestClient(make_server(app))
    import io
    buf = io.BytesIO()
    img.save(buf, format='PNG')
    r = client.post('/predict', content=buf.getvalue(), headers={'content-type': 'image/png'})
    assert r.status_code == 200 and r.headers['content-type'] == 'image/png'
    assert client.get('/metrics').status_code == 200
