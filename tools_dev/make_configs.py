"""Derive the BASELINE.json config variants from the stage-0 synthetic YAML (run once; output
committed under vfm-vae_amd/configs/). Every key not listed is the stage-0 reference value.
  python tools_dev/make_configs.py"""
import copy
import os

import yaml

HERE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vfm-vae_amd", "configs")
base = yaml.safe_load(open(os.path.join(HERE, "vfm_vae_f16d32_siglip2_stage_0_synthetic.yaml")))


def variant(name, header, edit):
    c = copy.deepcopy(base)
    edit(c)
    with open(os.path.join(HERE, name), "w") as f:
        f.write("".join(f"# {line}\n" for line in header.splitlines()))
        yaml.safe_dump(c, f, sort_keys=False, default_flow_style=None, width=110)


def c0(c):   # CLIP ViT-B/16 encoder, bs=1, CPU reconstruction
    c["run_dir"] = "runs/clip_b16_stage0_cpu"
    g = c["G_kwargs"]
    g.update(vfm_name="openai/clip-vit-base-patch16", scale_factor=1.0, patch_from_layers=[0, 6, -1],
             patch_in_dimensions=[768, 768, 768])
    c["batch_size"] = 1


def c3(c):   # DINOv2-L encoder, dynamic resolution 256/384/512
    c["run_dir"] = "runs/dinov2_l_dynres"
    g = c["G_kwargs"]
    g.update(vfm_name="facebook/dinov2-large", scale_factor=0.875, patch_from_layers=[0, 12, -1],
             patch_in_dimensions=[1024, 1024, 1024])
    c["training_set_kwargs"]["resolutions"] = [256, 384, 512]


def c4(c):   # discrete latent (VQ, 8 codebooks of 4096 x 4), fp16 decoder blocks
    c["run_dir"] = "runs/vq_f16d32"
    g = c["G_kwargs"]
    g.update(compression_mode="discrete", vocab_width=32, vocab_size=32768, num_codebooks=8, amp_dtype="float16")
    c["loss_kwargs"].update(compression_mode="discrete", kl_loss_weight=0.0, vq_loss_weight=1.0)


variant("vfm_vae_f16d32_clip_b16_stage_0_cpu.yaml",
        "BASELINE config 0: f16d32 stage 0 with a CLIP ViT-B/16 encoder (a build addition: the reference\n"
        "does not ship CLIP as an encoder), batch 1 at 256^2 -- the CPU plumbing case.", c0)
variant("vfm_vae_f16d32_dinov2_l_stage_0_dynres.yaml",
        "BASELINE config 3: DINOv2-L encoder (patch 14, scale 0.875 -> 16/24/32 patches) on a\n"
        "dynamic-resolution 256/384/512 stream (one size per micro-batch bucket).", c3)
variant("vfm_vae_f16d32_siglip2_stage_0_vq.yaml",
        "BASELINE config 4: discrete latent (VQ: vocab 32768 = 8 codebooks x 4096 of width 4) with fp16\n"
        "decoder blocks; codebook indices are bit-exact (vfm_codebook_argmax).", c4)
