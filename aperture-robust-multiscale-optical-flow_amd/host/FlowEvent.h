// FlowEvent.h — a flow result of the FARMS_Flow path.
//
// Same public interface as the reference's FlowEvent (/root/reference/include/
// FlowEvent.h:14-55): x, y, polarity, stamp, flow (Vx, Vy) and pooling scale.
// The reference's defects on this class are not reproduced (none of them reach
// its batch output): the constructor stores p, every setter
// returns true, and assignment assigns.
#ifndef FARMS_HOST_FLOWEVENT_H
#define FARMS_HOST_FLOWEVENT_H

class FlowEvent {
public:
    FlowEvent(int x, int y, double t, int p, double Vx, double Vy);
    FlowEvent();

    bool setX(int v);
    bool setY(int v);
    bool setStamp(double v);
    bool setPolarity(int v);
    bool setVx(double v);
    bool setVy(double v);
    bool setScale(int v);

    int getX() const;
    int getY() const;
    double getVx() const;
    double getVy() const;
    double getStamp() const;
    int getPolarity() const;
    int getScale() const;

private:
    int x_, y_, pol_;
    double t_, vx_, vy_;
    int scale_;
};

#endif
