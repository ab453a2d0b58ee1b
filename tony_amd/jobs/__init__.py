"""Reference jobs (the workloads of tony-examples), runnable through TonY.

| job | reference | runtime | parallelism |
|---|---|---|---|
| mnist_pytorch_ddp.py | EX/mnist-pytorch/mnist_distributed.py | pytorch | bucketed DDP all-reduce |
| mnist_tf_ps.py | EX/mnist-tensorflow/mnist_distributed.py | tensorflow | dedicated PS (async / sync) |
| mnist_tf_allreduce.py | EX/mnist-tensorflow/mnist_keras_distributed.py | tensorflow | MWMS-style all-reduce |
| mnist_estimator.py | EX/mnist-tensorflow/mnist_estimator_distributed.py | tensorflow | chief/worker/ps + evaluator |
| hvd_mnist.py | EX/horovod-on-tony/tensorflow2_mnist.py | horovod | hvd.DistributedOptimizer |
| hvd_resnet50.py | BASELINE.json ResNet-50 bf16 config | horovod | hvd.DistributedOptimizer |
| mxnet_linreg.py | EX/linearregression-mxnet/src/mxnet_dist_ex.py | mxnet | kvstore dist_sync / dist_async |
| inception_ps.py | BASELINE.json Inception-v3 TF-PS config | tensorflow | colocated / dedicated PS |
| cluster_discovery.py | EX/ray-on-tony/discovery.py | tensorflow | cluster-spec carrier |
"""
