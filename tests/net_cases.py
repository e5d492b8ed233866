"""Tiny-but-complete network configuration shared by the golden generator and
the parity tests (stage-0 structure at 64 px with a 2-layer SigLIP2 tower)."""

VFM_DIRNAME = "siglip2-tiny-patch16-64"
SIGLIP_CFG = dict(hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=4,
                  image_size=64, patch_size=16, num_channels=3)


def g_kwargs(vfm_dir, **over):
    kw = dict(
        vfm_name=vfm_dir, scale_factor=1.0, patch_from_layers=[0, 1, -1],
        patch_in_dimensions=[128, 128, 128], patch_out_dimensions=[64, 64, 64],
        compression_mode='continuous', how_to_compress='attnproj', how_to_decompress='attnproj',
        decompress_factor=16, attnproj_quant_layers=1, attnproj_post_quant_layers=1,
        resolution_compression_factor=16, z_dimension=32, z_pooled_resolution=1,
        z_dim_for_mapping_mlp_output=512, distmat_margin=0.0, cos_margin=0.0, distmat_weight=1.0, cos_weight=1.0,
        concat_z_block_indices=[0, 1, 2, 3], concat_z_mapped_dims=[512, 256, 128, 128],
        how_to_process_concat_z='unshuffle', activation_for_concat_z='lrelu',
        attn_block_indices=[0, 1, 2], attn_depths=[2, 2, 2], use_self_attn=True, use_cross_attn=False,
        use_convnext=True, use_gaussian_blur=True, add_additional_convnext=True,
        equivariance_regularization_p_prior=0.5, equivariance_regularization_p_prior_scale=0.25,
        num_blocks=6, num_fp16_res=3, train_mode='train_all', img_channels=3,
        synthesis_kwargs=dict(channel_base=32768, channel_max=512, num_res_blocks=2, architecture='skip'),
        legacy=True, img_resolution=64, conditional=False, label_type='cls2text',
        use_kl_loss=True, use_vf_loss=True, use_adaptive_vf_loss=True,
        use_equivariance_regularization=False, use_multiscale_output=True)
    kw.update(over)
    return kw


D_KWARGS = dict(vfm_name='siglip2', use_stylegan_t_discriminator=True, diffaug=False, p_crop=0.0,
                use_patchgan_discriminator=True, get_interm_feat=True)


def loss_kwargs(vfm_dir):
    return dict(vfm_name=vfm_dir, resume_kimg=0, use_equivariance_regularization=False, compression_mode='continuous',
                kl_loss_weight=1.0e-6, vf_loss_weight=5.0, use_adaptive_vf_loss=True, l1_pixel_loss_weight=1.0,
                l2_pixel_loss_weight=0.0, perceptual_loss_weight=10.0, ssim_loss_weight=0.0,
                multiscale_block_indices=[0, 1, 2, 3, 4], multiscale_pixel_loss_weights=[0.1] * 5,
                multiscale_pixel_loss_start_kimg=0, multiscale_pixel_loss_end_kimg=5000,
                stylegan_t_discriminator_loss_weight=1.0, patchgan_discriminator_loss_weight=1.0,
                feature_matching_loss_weight=10.0, use_stylegan_t_disc_warmup=False, use_patchgan_disc_warmup=False)
