// aiOS initramfs /init: a static, busybox-free early userspace (scripts/build-initramfs.sh).
//
// Steps (the same plan as the reference's busybox script, reference scripts/build-initramfs.sh):
//   1. mount proc / sysfs / devtmpfs
//   2. load the boot-path modules shipped in /lib/modules (finit_module)
//   3. find the boot medium: the block device whose filesystem label is AIOS (ISO 9660 volume id or ext4
//      label), else the first NVMe partition; mount it read-only
//   4. loop-mount /rootfs.squashfs (or /rootfs.ext4) from it, a tmpfs upper layer, overlay both at /newroot
//   5. aios.<key>=<value> kernel parameters -> AIOS_<KEY>=<value> in the environment
//   6. switch_root: move /newroot to /, chroot, exec /usr/sbin/aios-init (PID 1 stays PID 1)
// aios.debug_shell=1 or any failure execs /bin/sh when the image has one, else powers off after a delay.
//
// `init --plan` prints the steps it would take against the current machine without mounting anything
// (tests/test_distro.py runs it on the build host).
#define _GNU_SOURCE
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <linux/loop.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/mount.h>
#include <sys/reboot.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

static int plan_only = 0;

static void say(const char* fmt, const char* a, const char* b) {
  fprintf(stderr, "[aios-init-early] ");
  fprintf(stderr, fmt, a ? a : "", b ? b : "");
  fputc('\n', stderr);
}

static int do_mount(const char* src, const char* dst, const char* fs, unsigned long fl, const char* data) {
  if (plan_only) {
    fprintf(stdout, "mount -t %s %s %s%s%s\n", fs ? fs : "(bind)", src, dst, data ? " -o " : "", data ? data : "");
    return 0;
  }
  mkdir(dst, 0755);
  if (mount(src, dst, fs, fl, data) != 0) {
    say("mount %s failed: %s", dst, strerror(errno));
    return -1;
  }
  return 0;
}

static void rescue(void) {
  if (plan_only) exit(1);
  if (access("/bin/sh", X_OK) == 0) execl("/bin/sh", "sh", (char*)NULL);
  say("no rescue shell; powering off in 30 s%s%s", "", "");
  sleep(30);
  reboot(RB_POWER_OFF);
  _exit(1);
}

static void load_modules(void) {
  DIR* d = opendir("/lib/modules");
  if (!d) return;
  struct dirent* e;
  while ((e = readdir(d))) {
    if (!strstr(e->d_name, ".ko")) continue;
    char p[512];
    snprintf(p, sizeof p, "/lib/modules/%s", e->d_name);
    if (plan_only) {
      printf("insmod %s\n", p);
      continue;
    }
    int fd = open(p, O_RDONLY | O_CLOEXEC);
    if (fd < 0) continue;
    if (syscall(SYS_finit_module, fd, "", 0) != 0 && errno != EEXIST) say("insmod %s: %s", p, strerror(errno));
    close(fd);
  }
  closedir(d);
}

// filesystem label of a block device: ISO 9660 volume id (sector 16, offset 40) or ext2/3/4 (superblock
// at 1024, magic at +56, label at +120)
static int label_is(const char* dev, const char* want) {
  int fd = open(dev, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return 0;
  unsigned char buf[4096];
  int ok = 0;
  if (pread(fd, buf, 2048, 16 * 2048) == 2048 && memcmp(buf + 1, "CD001", 5) == 0) {
    char id[33];
    memcpy(id, buf + 40, 32);
    id[32] = 0;
    for (int i = 31; i >= 0 && id[i] == ' '; --i) id[i] = 0;
    ok = strcmp(id, want) == 0;
  } else if (pread(fd, buf, 1024, 1024) == 1024 && buf[56] == 0x53 && buf[57] == 0xEF) {
    char id[17];
    memcpy(id, buf + 120, 16);
    id[16] = 0;
    ok = strcmp(id, want) == 0;
  }
  close(fd);
  return ok;
}

static int find_medium(char* out, size_t n) {
  for (int tries = 0; tries < 30; ++tries) {
    DIR* d = opendir("/sys/class/block");
    if (d) {
      struct dirent* e;
      while ((e = readdir(d))) {
        if (e->d_name[0] == '.') continue;
        char dev[300];
        snprintf(dev, sizeof dev, "/dev/%s", e->d_name);
        if (label_is(dev, "AIOS")) {
          snprintf(out, n, "%s", dev);
          closedir(d);
          return 0;
        }
      }
      closedir(d);
    }
    if (plan_only) break;
    usleep(500 * 1000);
  }
  snprintf(out, n, "/dev/nvme0n1p1");
  return access(out, F_OK) == 0 || plan_only ? 0 : -1;
}

static int loop_attach(const char* file, char* dev, size_t n) {
  if (plan_only) {
    snprintf(dev, n, "/dev/loopN");
    printf("losetup -r %s %s\n", dev, file);
    return 0;
  }
  int ctl = open("/dev/loop-control", O_RDWR | O_CLOEXEC);
  if (ctl < 0) return -1;
  int idx = ioctl(ctl, LOOP_CTL_GET_FREE);
  close(ctl);
  if (idx < 0) return -1;
  snprintf(dev, n, "/dev/loop%d", idx);
  int lfd = open(dev, O_RDWR | O_CLOEXEC), ffd = open(file, O_RDONLY | O_CLOEXEC);
  if (lfd < 0 || ffd < 0) return -1;
  struct loop_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.fd = (unsigned)ffd;
  cfg.info.lo_flags = LO_FLAGS_READ_ONLY | LO_FLAGS_AUTOCLEAR;
  int r = ioctl(lfd, LOOP_CONFIGURE, &cfg);
  close(ffd);
  close(lfd);
  return r;
}

// aios.<key>=<value> -> AIOS_<KEY>=<value> ('.' -> '_', upper case)
static void export_cmdline(int* debug_shell) {
  char buf[4096] = {0};
  FILE* f = fopen("/proc/cmdline", "r");
  if (!f) return;
  size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  for (char* tok = strtok(buf, " \n"); tok; tok = strtok(NULL, " \n")) {
    if (strncmp(tok, "aios.", 5) != 0) continue;
    char* eq = strchr(tok, '=');
    if (!eq) continue;
    char key[256] = "AIOS_";
    size_t k = 5;
    for (char* p = tok + 5; p < eq && k < sizeof key - 1; ++p) key[k++] = *p == '.' ? '_' : (char)(*p >= 'a' && *p <= 'z' ? *p - 32 : *p);
    key[k] = 0;
    if (strcmp(key, "AIOS_DEBUG_SHELL") == 0 && strcmp(eq + 1, "1") == 0) *debug_shell = 1;
    if (plan_only) printf("export %s=%s\n", key, eq + 1);
    else setenv(key, eq + 1, 1);
  }
}

int main(int argc, char** argv) {
  plan_only = argc > 1 && strcmp(argv[1], "--plan") == 0;
  if (!plan_only) {
    do_mount("proc", "/proc", "proc", 0, NULL);
    do_mount("sysfs", "/sys", "sysfs", 0, NULL);
    do_mount("devtmpfs", "/dev", "devtmpfs", 0, NULL);
  } else {
    printf("mount -t proc proc /proc\nmount -t sysfs sysfs /sys\nmount -t devtmpfs devtmpfs /dev\n");
  }
  load_modules();
  char medium[300], loop[64];
  if (find_medium(medium, sizeof medium) != 0) rescue();
  if (do_mount(medium, "/mnt/medium", "iso9660", MS_RDONLY, NULL) != 0 &&
      do_mount(medium, "/mnt/medium", "ext4", MS_RDONLY, NULL) != 0)
    rescue();
  // the root image: rootfs.squashfs, else an ext4 image (rootfs.ext4: what mkfs.ext4 -d packs on a
  // build host without squashfs tools), mounted read-only either way
  const char *img = "/mnt/medium/rootfs.squashfs", *img_fs = "squashfs";
  if (!plan_only && access(img, F_OK) != 0) {
    img = "/mnt/medium/rootfs.ext4";
    img_fs = "ext4";
  }
  if (loop_attach(img, loop, sizeof loop) != 0) rescue();
  if (do_mount(loop, "/mnt/ro", img_fs, MS_RDONLY, NULL) != 0) rescue();
  if (do_mount("tmpfs", "/mnt/rw", "tmpfs", 0, "mode=0755") != 0) rescue();
  if (!plan_only) {
    mkdir("/mnt/rw/upper", 0755);
    mkdir("/mnt/rw/work", 0755);
  }
  if (do_mount("overlay", "/newroot", "overlay", 0, "lowerdir=/mnt/ro,upperdir=/mnt/rw/upper,workdir=/mnt/rw/work") != 0)
    rescue();
  int debug_shell = 0;
  export_cmdline(&debug_shell);
  if (debug_shell) rescue();
  if (plan_only) {
    printf("switch_root /newroot /usr/sbin/aios-init\n");
    return 0;
  }
  // switch_root: the overlay becomes /, the initramfs contents stay unreachable (freed with the rootfs)
  if (chdir("/newroot") != 0 || mount("/newroot", "/", NULL, MS_MOVE, NULL) != 0 || chroot(".") != 0 || chdir("/") != 0)
    rescue();
  execl("/usr/sbin/aios-init", "aios-init", (char*)NULL);
  say("exec /usr/sbin/aios-init: %s%s", strerror(errno), "");
  rescue();
  return 1;
}
