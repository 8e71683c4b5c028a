from .deeplab_multi import DeeplabMulti, ResNetMulti, Bottleneck, Classifier_Module  # noqa: F401
from .discriminator import FCDiscriminator  # noqa: F401
from .deeplab_vgg import DeeplabVGG  # noqa: F401
from .warper import Warper  # noqa: F401
