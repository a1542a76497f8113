"""Host-side profile of the BERT-base training step (cProfile, 10 steps after warm-up)."""
import cProfile, os, pstats, sys, io
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "analytics-zoo_amd"))
sys.argv = ["bert_train.py", "--batch", "128", "--iters", "10"]
import importlib.util
spec = importlib.util.spec_from_file_location("bt", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                                                  "analytics-zoo_amd", "tools", "bert_train.py"))
bt = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bt)
pr = cProfile.Profile()
pr.enable()
bt.main()
pr.disable()
s = io.StringIO()
ps = pstats.Stats(pr, stream=s).sort_stats("tottime")
ps.print_stats(35)
print(s.getvalue()[:9000])
