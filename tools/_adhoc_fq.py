import ctypes, os, sys, statistics, torch
sys.path.insert(0, "mi-bminet_amd")
from mibminet.params import ParamSet
blob = ParamSet.synthetic(seed=1).to_blob()
libs = []
for p in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(p), mode=ctypes.RTLD_LOCAL)
    L.net_params_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    L.net_model_compute_batch_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
    assert L.net_params_load(blob, len(blob)) == 0
    libs.append(L)
x = torch.randn((65536, 22, 1125), dtype=torch.float32, device="cuda") * 50
y = torch.empty((65536, 4), dtype=torch.int8, device="cuda")
st = torch.cuda.current_stream()
outs = []
for L in libs:
    L.net_model_compute_batch_f32(x.data_ptr(), y.data_ptr(), 65536, 200.0, 0, st.cuda_stream); torch.cuda.synchronize(); outs.append(y.clone())
print("same outputs:", all(torch.equal(o, outs[0]) for o in outs))
t = {p: [] for p in sys.argv[1:]}
for r in range(6):
    for p, L in zip(sys.argv[1:], libs):
        for _ in range(2): L.net_model_compute_batch_f32(x.data_ptr(), y.data_ptr(), 65536, 200.0, 0, st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10): L.net_model_compute_batch_f32(x.data_ptr(), y.data_ptr(), 65536, 200.0, 0, st.cuda_stream)
        e1.record(st); e1.synchronize()
        t[p].append(e0.elapsed_time(e1) / 10)
for p in t: print(os.path.basename(p), round(statistics.median(t[p]), 4))
