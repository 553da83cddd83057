"""distributed_llms_example_amd — MI355X-native distributed seq2seq fine-tuning.

Layers (see README.md / SURVEY.md §7): ``ops`` (HIP kernel library + references), ``models``
(T5 / FLAN-T5 / BART, HF-compatible I/O), ``parallel`` (process bootstrap, flat params, bucketed
RCCL gradient reducer, samplers, collectives), ``data`` (SAMSum JSON, synthetic, collator),
``train`` (Trainer-style and Accelerate-style loops, schedules, checkpoints, ROUGE, callbacks),
``platform`` (Valohai paths/metadata), ``utils`` (logging, GPU report, timers).
"""
__version__ = "0.1.0"
