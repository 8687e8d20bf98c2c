import cProfile, pstats, os, sys, io
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from tomatis_audio_processor_amd import engine
ss = engine.StreamSet.synthetic(64, 300 * 44100, 2, 44100, seed0=1000)
G = int(os.environ.get('TOMATIS_C3_GROUPS', '0'))
pipe = engine.AdaptiveGroups(ss, groups=G, n_fft=2048, hop=512) if G else engine.AdaptivePipeline(ss, n_fft=2048, hop=512)
pipe.run(); torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    pipe.run()
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
print(s.getvalue())
