"""Hyper-parameter dicts of the reference (config.py), same names and values.

Only `G`, `D` and `loss` feed the hot path (the G+D train step, tpgan_train.py); the
pretraining dicts are kept so that `from config import ...` lines of callers resolve.
"""
pretrain = dict(
    txt_name="list_landmarks_celeba.txt",
    data_root_dir="C:\\Users\\User\\Downloads\\CelebA",
    log_root_dir="C:\\Users\\User\\Desktop\\Test\\SummaryWriterLog",
    model_name="MobileNetV2",
    train_data_ratio=0.95,
    validation_data_ratio=0.0005,
    batch_size=1,
    optimizer="SGD",
    use_learning_rate_scheduler=True,
    learning_rate_scheduler_milestone=[10, 20, 30],
    learning_rate_scheduler_gamma=0.1,
    num_epochs=5,
    log_step_of_batchs=200,
    loss=dict(alpha=30.0, beta=0.1, ratio_non_background=5.0),
)

optimizer_param = dict(learning_rate=5e-4, momentum=0.9, nesterov=True, weight_decay=5e-4)

general = dict(image_max_size=1024)

# The reference marks everything below as provisional (config.py:48).
train = dict(img_list="./img.list", learning_rate=1e-4, num_epochs=50, batch_size=50, log_step=1000,
             resume_model=None, resume_optimizer=None)

G = dict(zdim=64, use_residual_block=False, use_batchnorm=False, num_classes=347)

D = dict(use_batchnorm=False)

loss = dict(
    weight_gradient_penalty=10,
    weight_128=1.0,
    weight_64=1.0,
    weight_32=1.5,
    weight_pixelwise=1.0,
    weight_pixelwise_local=3.0,
    weight_symmetry=3e-1,
    weight_adv_G=1e-3,
    weight_identity_preserving=3e1,
    weight_total_varation=1e-3,
    weight_cross_entropy=1e1,
)

feature_extract_model = dict(resume="save/feature_extract_model/resnet18/try_1")
