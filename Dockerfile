# MI355X (gfx950) image: ROCm 7.2 + PyTorch-ROCm; the HIP kernel library is compiled for gfx950 at build time.
FROM rocm/pytorch:rocm7.2_ubuntu22.04_py3.10_pytorch_release_2.10.0

ENV HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTORCH_ROCM_ARCH=gfx950 \
    PYTHONUNBUFFERED=1

RUN pip install --no-cache-dir "transformers>=4.46" safetensors tokenizers sentencepiece valohai-utils pyyaml

WORKDIR /workspace
COPY . /workspace
RUN python tools/build_native.py --force && python -c "import distributed_llms_example_amd._C as C; print(C.arch)"
